#!/bin/bash
# Round 4, batch 16: at C3 the LW chain now ends last; both networks confined to complementary parts of the chip and
# started together (the SW network on the larger part, the critical path), against the default (LW chain after the SW
# network, LW network on 160 CUs); whole steps, alternating.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
CASES="default|default|
split64|default|--lw-after none --lw-net-cus 64 --sw-net-cus 192
split96|default|--lw-after none --lw-net-cus 96 --sw-net-cus 160
split128|default|--lw-after none --lw-net-cus 128 --sw-net-cus 128" CONFIGS="c3" REPS=3 STEPS=50 timeout -k 10 600 bash tools/gpu_ab.sh > gpurun_out/r04/split_c3.txt 2>&1
rc=$?; cat gpurun_out/r04/split_c3.txt; exit $rc
