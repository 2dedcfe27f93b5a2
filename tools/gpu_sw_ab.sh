#!/bin/bash
# SW solver A/B on one box: parity of every SW kernel mode, then bench lines of mode 2 (two per lane) against mode 3
# (checkpointed) for the default build and the variants/ builds.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_clouds.py tests/test_gpu_glue.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sw.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_sw.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for cfg in ${CONFIGS:-c3 c4}; do for rep in 1 2; do for lib in default ${VARIANTS:-}; do for k in 2 3; do
  if [ $lib = default ]; then L=""; else L="RRTMGPNN_LIB=$PWD/variants/$lib.so"; fi
  env $L timeout -k 10 300 python bench.py --config $cfg --steps 50 --warmup 5 --no-cpu-baseline --sw-kernel $k > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$cfg $lib sw$k', round(d['value']), d['ms_per_step'], d['stages_ms']['sw_solver'], d['stages_overlapped_ms']['sw_solver'])"
done; done; done; done
