#!/bin/bash
# GPU suite, then an alternating A/B of the LW MLP tiling (RRTMGPNN_MLP32=1: 32x32x2 kernel, 0: 16x16x4 kernel) on
# whole C3/C4 bench lines with their serialised stage times.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for cfg in ${CONFIGS:-c3 c4}; do for rep in 1 2; do for v in ${VALS:-1 0}; do
  RRTMGPNN_MLP32=$v timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-50} --warmup 5 --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$cfg mlp32=$v', round(d['value']), d['ms_per_step'], d['stages_ms'].get('predict_nn_lw'), d['stages_overlapped_ms'].get('predict_nn_lw'))"
done; done; done
