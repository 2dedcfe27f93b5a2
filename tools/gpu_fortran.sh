#!/bin/bash
# Fortran drop-in on the GPU: its tests, then the C3 block loop through rrtmgpnn_rfmip_clear_sky at several
# block sizes / thread counts beside the Python pipeline's bench line.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fortran.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_fortran.log 2>&1
rc=$?; tail -n 12 gpurun_out/pytest_fortran.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --c5-steps 0 > gpurun_out/fb_py.json 2> gpurun_out/fb_py.err || { tail -5 gpurun_out/fb_py.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/fb_py.json')); print('python pipeline', d['value'], d['ms_per_step'], 'host_resident', d['host_resident'])"
for cfg in "1800 1" "900 2" "600 3" "450 4" "225 8"; do set -- $cfg
  timeout -k 10 300 python bench.py --fortran --fortran-block $1 --fortran-threads $2 --steps 50 > gpurun_out/fb_$1_$2.json 2> gpurun_out/fb.err || { tail -5 gpurun_out/fb.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/fb_$1_$2.json')); print('fortran block $1 threads $2', d['value'], d['ms_per_step'])"
done
