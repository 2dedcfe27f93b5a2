#!/bin/bash
# Quick GPU iteration: full GPU test suite, then C3 and C4 bench lines (no CPU baseline). Stops at the first failure.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for cfg in ${CONFIGS:-c3 c4}; do
  timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err || { rc=$?; tail -5 gpurun_out/bench_$cfg.err; exit $rc; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/bench_$cfg.json')); print('$cfg', d['value'], d['ms_per_step'], d['stages_ms'])"
done
