#!/bin/bash
# Round 4, batch 10: the default step schedule (LW chain after the SW network) with the SW stream at high priority,
# so that the SW solver's blocks are dispatched ahead of the LW network's when both become ready; C3 and C4 whole
# steps, alternating.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
CASES="gate|default|
gate_prio|default|--sw-priority -1
together_prio|default|--lw-after none --sw-priority -1" CONFIGS="c3 c4" REPS=3 STEPS=50 timeout -k 10 900 bash tools/gpu_ab.sh > gpurun_out/r04/prio_b10.txt 2>&1
rc=$?; cat gpurun_out/r04/prio_b10.txt; exit $rc
