#!/bin/bash
# rocprofv3 runtime trace (HIP API + kernels + copies) of the Fortran drop-in's C3 block loop at several
# (block size, OpenMP threads) settings: gpurun_out/fprof_<block>_<threads>/ (CFGS="900 2;450 4" by default)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
python3 - <<'PY'
import sys; sys.path.insert(0, "rte-rrtmgp-nn_amd")
from rrtmgpnn import data
data.write_problem(data.rfmip_columns(0, 1800), "gpurun_out/c3_problem.rbin")
PY
IFS=';' read -ra CF <<< "${CFGS:-1800 1;900 2;450 4}"
for cfg in "${CF[@]}"; do set -- $cfg
  OMP_NUM_THREADS=$2 timeout -k 10 300 rocprofv3 --runtime-trace --stats -d gpurun_out/fprof_$1_$2 -o run --output-format csv -- rte-rrtmgp-nn_amd/fortran/build/rrtmgpnn_rfmip_clear_sky gpurun_out/c3_problem.rbin gpurun_out/f_out.rbin rte-rrtmgp-nn_amd/data $1 21 > gpurun_out/fprof_$1_$2.log 2>&1 || { tail -5 gpurun_out/fprof_$1_$2.log; exit 1; }
  grep timing gpurun_out/fprof_$1_$2.log
  ms=$(grep -o "timing: *[0-9.]*" gpurun_out/fprof_$1_$2.log | grep -o "[0-9.]*$")
  python3 tools/trace_threads.py gpurun_out/fprof_$1_$2 $ms 10 | tee gpurun_out/fprof_$1_$2.summary
done
rm -f gpurun_out/c3_problem.rbin gpurun_out/f_out.rbin
