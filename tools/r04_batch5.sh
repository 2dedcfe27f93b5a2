#!/bin/bash
# Round 4, batch 5: the whole -m gpu suite on the round's build, the C4 schedules, then the profile set of C3 and C4
# (tools/profile_configs.sh: kernel traces overlapped and --no-overlap, PMC traffic, SQ and MFMA counters, the bench
# line with them).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/r04/pytest_gpu_b5.log 2>&1
rc=$?; tail -2 gpurun_out/r04/pytest_gpu_b5.log; [ $rc -eq 0 ] || exit $rc
CASES="together|default|
nets_first|default|--sw-after predict_nn_lw" CONFIGS="c4" REPS=2 STEPS=30 timeout -k 10 600 bash tools/gpu_ab.sh > gpurun_out/r04/sched_c4.txt 2>&1
rc=$?; cat gpurun_out/r04/sched_c4.txt; [ $rc -eq 0 ] || exit $rc
CONFIGS="c3 c4" bash tools/profile_configs.sh
