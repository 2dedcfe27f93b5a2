#!/bin/bash
# Round 4: SW network occupancy variants (block size, waves-per-SIMD floor) -- the network alone (bitwise), then C3
# steps; plus the default build's bench line (settled and unsettled) for the record.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
V="variants/mlp_sw512w4.so variants/mlp_sw256w3.so variants/mlp_sw256w4.so"
for c in c3 c4; do
  timeout -k 10 300 python -u tools/kernel_ab.py --config $c --stage predict_nn_sw --rounds 9 --iters 20 $V > gpurun_out/r04/mlpsw_$c.txt 2>&1 || { tail -5 gpurun_out/r04/mlpsw_$c.txt; exit 1; }
  grep predict_nn_sw gpurun_out/r04/mlpsw_$c.txt
done
CASES="base|default|
sw512w4|variants/mlp_sw512w4.so|
sw256w3|variants/mlp_sw256w3.so|
sw256w4|variants/mlp_sw256w4.so|" CONFIGS="c3" REPS=2 STEPS=50 timeout -k 10 600 bash tools/gpu_ab.sh > gpurun_out/r04/mlpsw_step.txt 2>&1
rc=$?; cat gpurun_out/r04/mlpsw_step.txt; [ $rc -eq 0 ] || exit $rc
# the small SW solver instance at a 4-wave floor (one round of residency at C3), K = 3 / ring 6 and K = 2 / ring 6
timeout -k 10 300 python -u tools/kernel_ab.py --config c3 --stage sw_solver --rounds 9 --iters 20 variants/sw_k3r6w4.so variants/sw_k2r6w4.so > gpurun_out/r04/sww4_c3.txt 2>&1 || { tail -5 gpurun_out/r04/sww4_c3.txt; exit 1; }
grep sw_solver gpurun_out/r04/sww4_c3.txt
