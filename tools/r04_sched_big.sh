#!/bin/bash
# Round 4: the LW-after-SW-network gate at large grids (C4 all-sky, C5 shard) against the chains started together
# (the default there), whole steps alternating.  At C4 the SW chain is the critical path: started together, the SW
# network runs beside the LW network and the LW solver (775 us against 237 alone) and the SW solver starts late.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
CASES="together|default|--lw-after none
lw_gate|default|--lw-after predict_nn_sw" CONFIGS="c4" REPS=3 STEPS=30 timeout -k 10 600 bash tools/gpu_ab.sh > gpurun_out/r04/sched_big_c4.txt 2>&1
rc=$?; cat gpurun_out/r04/sched_big_c4.txt; [ $rc -eq 0 ] || exit $rc
CASES="together|default|--lw-after none
lw_gate|default|--lw-after predict_nn_sw" CONFIGS="c5" REPS=2 STEPS=10 timeout -k 10 900 bash tools/gpu_ab.sh > gpurun_out/r04/sched_big_c5.txt 2>&1
rc=$?; cat gpurun_out/r04/sched_big_c5.txt; exit $rc
