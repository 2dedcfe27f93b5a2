#!/bin/bash
# Round 4, batch 7 (the LW gate back as the C3 default): the schedule-dependent tests, the C3 and C5 profile sets
# (tools/profile_configs.sh), then the driver's own bench command with the CPU baseline.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_chunked.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/r04/pytest_b7.log 2>&1
rc=$?; tail -2 gpurun_out/r04/pytest_b7.log; [ $rc -eq 0 ] || exit $rc
CONFIGS="c3" bash tools/profile_configs.sh || exit $?
STEPS=10 CONFIGS="c5" bash tools/profile_configs.sh || exit $?
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04/bench_driver_cmd.json 2> gpurun_out/r04/bench_driver_cmd.err
rc=$?; head -c 600 gpurun_out/r04/bench_driver_cmd.json; exit $rc
