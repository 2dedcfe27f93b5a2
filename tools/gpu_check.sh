#!/bin/bash
# One GPU-box session: parity tests, a short bench, a rocprofv3 kernel-trace summary.
# Stops at the first fault/abort/timeout (exit codes other than 0/1), per the pool's rules.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-30}
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
echo "== pytest -m gpu" 
timeout -k 10 ${PYTEST_TIMEOUT:-600} python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
echo "== bench"
timeout -k 10 300 python bench.py --steps $STEPS --warmup 5 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
ok $rc || exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  echo "== rocprofv3 kernel trace"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps $STEPS --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof.log
  find gpurun_out/prof -name "*stats*" | head
fi
exit 0
