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
timeout -k 10 300 python bench.py --steps $STEPS --warmup 5 ${BENCH_ARGS:-} --c5-steps 0 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
ok $rc || exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  echo "== rocprofv3 kernel trace"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps $STEPS --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} --c5-steps 0 > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof.log
  [ $rc -eq 0 ] || exit $rc
  find gpurun_out/prof -name "*stats*" | head
fi
if [ "${PMC:-0}" = "1" ]; then
  # HBM bytes per launch: FETCH_SIZE and WRITE_SIZE in separate passes (MI355X_MICROARCH.md, HBM section)
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "== rocprofv3 --pmc $c"
    timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/pmc_$c -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-graph ${BENCH_ARGS:-} --c5-steps 0 > gpurun_out/pmc_$c.log 2>&1
    rc=$?; echo "pmc $c rc=$rc"; tail -2 gpurun_out/pmc_$c.log
    [ $rc -eq 0 ] || exit $rc
  done
  python3 tools/pmc_traffic.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE ${CONFIG:-c3} gpurun_out/pmc_traffic.json
fi
exit 0
