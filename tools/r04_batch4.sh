#!/bin/bash
# Round 4, batch 4: the fused LW down pass reusing its neighbour's Planck fraction (parity, then alone against the
# previous build), step schedules, the SW network's occupancy variants and the 4-wave SW solver instance.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_gpt.py -x -q --timeout 240 --timeout-method thread -rf > gpurun_out/r04/pytest_b4.log 2>&1
rc=$?; tail -2 gpurun_out/r04/pytest_b4.log; [ $rc -eq 0 ] || exit $rc
for c in c3 c4; do
  timeout -k 10 300 python -u tools/kernel_ab.py --config $c --stage lw_solver --rounds 9 --iters 10 variants/lw_pvload.so > gpurun_out/r04/lwpv_$c.txt 2>&1 || { tail -5 gpurun_out/r04/lwpv_$c.txt; exit 1; }
  grep lw_solver gpurun_out/r04/lwpv_$c.txt
done
CASES="gate|default|
nets_first_prio|default|--lw-after none --sw-after predict_nn_lw --sw-priority -1
nets_first|default|--lw-after none --sw-after predict_nn_lw
together|default|--lw-after none" CONFIGS="c3" REPS=3 STEPS=50 timeout -k 10 900 bash tools/gpu_ab.sh > gpurun_out/r04/sched_step.txt 2>&1
rc=$?; cat gpurun_out/r04/sched_step.txt; [ $rc -eq 0 ] || exit $rc
bash tools/r04_mlpsw.sh
