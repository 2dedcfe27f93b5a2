#!/bin/bash
# Round 4: staggered ring-flush phases (SW checkpointed and LW no-scattering solvers) -- solver parity tests, then
# each solver alone against the unstaggered builds (bitwise), then whole C3 / C4 steps.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_gpt.py tests/test_gpu_lw_scat.py tests/test_gpu_clouds.py -x -q --timeout 240 --timeout-method thread -rf > gpurun_out/r04/pytest_stagger.log 2>&1
rc=$?; tail -3 gpurun_out/r04/pytest_stagger.log; [ $rc -eq 0 ] || exit $rc
for c in c3 c4; do
  timeout -k 10 300 python -u tools/kernel_ab.py --config $c --stage sw_solver --rounds 7 --iters 10 variants/sw_nostagger.so > gpurun_out/r04/stagger_sw_$c.txt 2>&1 || { tail -5 gpurun_out/r04/stagger_sw_$c.txt; exit 1; }
  grep sw_solver gpurun_out/r04/stagger_sw_$c.txt
  timeout -k 10 300 python -u tools/kernel_ab.py --config $c --stage lw_solver --rounds 7 --iters 10 variants/lw_nostagger.so > gpurun_out/r04/stagger_lw_$c.txt 2>&1 || { tail -5 gpurun_out/r04/stagger_lw_$c.txt; exit 1; }
  grep lw_solver gpurun_out/r04/stagger_lw_$c.txt
done
CASES="stagger|default|
nostagger|variants/nostagger.so|" CONFIGS="c3 c4" REPS=3 STEPS=50 timeout -k 10 900 bash tools/gpu_ab.sh > gpurun_out/r04/stagger_step.txt 2>&1
rc=$?; cat gpurun_out/r04/stagger_step.txt; exit $rc
