#!/bin/bash
# Round 4, batch 11: the all-sky SW solver with one band value per lane (both g-points of a lane in one band) --
# C4 SW solver alone against the default build (bitwise), then C4 whole steps.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u tools/kernel_ab.py --config c4 --stage sw_solver --rounds 9 --iters 10 variants/bandpair.so > gpurun_out/r04/bandpair_c4.txt 2>&1 || { tail -5 gpurun_out/r04/bandpair_c4.txt; exit 1; }
grep sw_solver gpurun_out/r04/bandpair_c4.txt
CASES="base|default|
bandpair|variants/bandpair.so|" CONFIGS="c4" REPS=3 STEPS=30 timeout -k 10 600 bash tools/gpu_ab.sh > gpurun_out/r04/bandpair_step.txt 2>&1
rc=$?; cat gpurun_out/r04/bandpair_step.txt; exit $rc
