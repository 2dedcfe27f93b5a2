#!/bin/bash
# Round 4, final build with the LW-network CU cap at small grids: the whole -m gpu suite, smoke(), the C3 profile set,
# the driver's bench command (with the CPU baseline) and the self-launched two-rank line.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/r04/pytest_final2.log 2>&1
rc=$?; tail -2 gpurun_out/r04/pytest_final2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04/smoke_final2.log 2>&1
rc=$?; tail -1 gpurun_out/r04/smoke_final2.log; [ $rc -eq 0 ] || exit $rc
CONFIGS="c3" bash tools/profile_configs.sh || exit $?
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04/bench_driver_final2.json 2> gpurun_out/r04/bench_driver_final2.err
rc=$?; head -c 300 gpurun_out/r04/bench_driver_final2.json; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04/bench_n2_final2.json 2> gpurun_out/r04/bench_n2_final2.err
rc=$?; head -c 300 gpurun_out/r04/bench_n2_final2.json; echo; exit $rc
