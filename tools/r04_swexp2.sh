#!/bin/bash
# Round 4 SW-solver experiment 2: combinations of the fence-free walk with the small-grid instance's chunk length,
# ring, wave floor and workspace planes (kernel alone, bitwise against the default), then whole C3 steps.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
V=$(ls variants/*.so)
timeout -k 10 300 python -u tools/kernel_ab.py --config c3 --stage sw_solver --rounds 11 --iters 20 $V > gpurun_out/r04/swexp2_c3.txt 2>&1 || { tail -5 gpurun_out/r04/swexp2_c3.txt; exit 1; }
grep sw_solver gpurun_out/r04/swexp2_c3.txt
CASES="base|default|
nofence|variants/nofence.so|
nf_k3|variants/nf_k3.so|" CONFIGS=c3 REPS=3 STEPS=50 timeout -k 10 600 bash tools/gpu_ab.sh > gpurun_out/r04/swexp2_step.txt 2>&1
rc=$?; cat gpurun_out/r04/swexp2_step.txt; exit $rc
