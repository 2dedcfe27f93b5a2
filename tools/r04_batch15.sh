#!/bin/bash
# Round 4, batch 15: around the default LW-network cap at C3 (160 CUs): 128 and 144 CUs, and with the cap the chains
# started together instead of the LW chain after the SW network; whole steps, alternating.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
CASES="cus160|default|
cus128|default|--lw-net-cus 128
cus144|default|--lw-net-cus 144
together160|default|--lw-after none --lw-net-cus 160" CONFIGS="c3" REPS=3 STEPS=50 timeout -k 10 600 bash tools/gpu_ab.sh > gpurun_out/r04/lwcus2_c3.txt 2>&1
rc=$?; cat gpurun_out/r04/lwcus2_c3.txt; exit $rc
