#!/bin/bash
# Round 4: step schedules at C3 (whole steps, alternating): the default gate (LW chain after the SW network), both
# networks first and then the two solvers side by side (with and without a high-priority SW stream), both chains
# started together.  Then the overlap parity test that covers these schedules.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py -x -q -k overlap --timeout 240 --timeout-method thread -rf > gpurun_out/r04/pytest_sched.log 2>&1
rc=$?; tail -2 gpurun_out/r04/pytest_sched.log; [ $rc -eq 0 ] || exit $rc
CASES="gate|default|
nets_first_prio|default|--lw-after none --sw-after predict_nn_lw --sw-priority -1
nets_first|default|--lw-after none --sw-after predict_nn_lw
together|default|--lw-after none" CONFIGS="c3" REPS=3 STEPS=50 timeout -k 10 900 bash tools/gpu_ab.sh > gpurun_out/r04/sched_step.txt 2>&1
rc=$?; cat gpurun_out/r04/sched_step.txt; exit $rc
