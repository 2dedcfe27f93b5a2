#!/bin/bash
# Round 4, batch 13: the LW network on fewer CUs at C3 (grid capped at 192 or 128 one-per-CU blocks), so that SW
# solver blocks start on the other CUs at once instead of after the LW network's 75 us; whole C3 steps, alternating.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
CASES="base|default|
lwgrid192|variants/lwgrid192.so|
lwgrid128|variants/lwgrid128.so|" CONFIGS="c3" REPS=3 STEPS=50 timeout -k 10 900 bash tools/gpu_ab.sh > gpurun_out/r04/lwgrid_step.txt 2>&1
rc=$?; cat gpurun_out/r04/lwgrid_step.txt; exit $rc
