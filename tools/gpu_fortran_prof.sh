#!/bin/bash
# rocprofv3 runtime trace (HIP API + kernels) of the Fortran drop-in's C3 block loop.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
python3 - <<'PY'
import sys; sys.path.insert(0, "rte-rrtmgp-nn_amd")
from rrtmgpnn import data
data.write_problem(data.rfmip_columns(0, 1800), "gpurun_out/c3_problem.rbin")
PY
for cfg in "1800 1" "900 2"; do set -- $cfg
  OMP_NUM_THREADS=$2 timeout -k 10 300 rocprofv3 --runtime-trace --stats -d gpurun_out/fprof_$1 -o run --output-format csv -- rte-rrtmgp-nn_amd/fortran/build/rrtmgpnn_rfmip_clear_sky gpurun_out/c3_problem.rbin gpurun_out/f_out.rbin rte-rrtmgp-nn_amd/data $1 6 > gpurun_out/fprof_$1.log 2>&1 || { tail -5 gpurun_out/fprof_$1.log; exit 1; }
  grep timing gpurun_out/fprof_$1.log
done
rm -f gpurun_out/c3_problem.rbin gpurun_out/f_out.rbin
