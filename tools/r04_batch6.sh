#!/bin/bash
# Round 4, batch 6: the whole -m gpu suite (the SW solver now waits for both networks), the step schedules at C3 and
# C4 (both networks first then the solvers side by side; the LW chain after the SW network; both chains together),
# then the profile set of C3 and C4 (tools/profile_configs.sh).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/r04/pytest_gpu_b6.log 2>&1
rc=$?; tail -2 gpurun_out/r04/pytest_gpu_b6.log; [ $rc -eq 0 ] || exit $rc
CASES="nets_first|default|--lw-after none --sw-after predict_nn_lw
lw_gate|default|--lw-after predict_nn_sw --sw-after none
together|default|--lw-after none --sw-after none" CONFIGS="c3 c4" REPS=3 STEPS=50 timeout -k 10 900 bash tools/gpu_ab.sh > gpurun_out/r04/sched_b6.txt 2>&1
rc=$?; cat gpurun_out/r04/sched_b6.txt; [ $rc -eq 0 ] || exit $rc
CONFIGS="c3 c4" bash tools/profile_configs.sh
