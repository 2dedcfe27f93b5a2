#!/bin/bash
# Round 4, batch 12: the LW network reading its per-input arguments from the kernel-argument segment at each tile
# (no SGPR spills) -- the LW network alone at C3 and C4 against the default build (bitwise), then C3 whole steps.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
for c in c3 c4; do
  timeout -k 10 300 python -u tools/kernel_ab.py --config $c --stage predict_nn_lw --rounds 9 --iters 20 variants/mlpka.so > gpurun_out/r04/mlpka_$c.txt 2>&1 || { tail -5 gpurun_out/r04/mlpka_$c.txt; exit 1; }
  grep predict_nn_lw gpurun_out/r04/mlpka_$c.txt
done
CASES="base|default|
mlpka|variants/mlpka.so|" CONFIGS="c3" REPS=3 STEPS=50 timeout -k 10 600 bash tools/gpu_ab.sh > gpurun_out/r04/mlpka_step.txt 2>&1
rc=$?; cat gpurun_out/r04/mlpka_step.txt; exit $rc
