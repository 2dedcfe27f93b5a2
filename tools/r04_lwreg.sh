#!/bin/bash
# Round 4: the LW register-resident up pass -- its parity tests first, then the LW solver alone against the
# recompute kernel and other register budgets (tools/kernel_ab.py, bitwise), then whole C3 steps.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -rf > gpurun_out/r04/pytest_lwreg.log 2>&1
rc=$?; tail -3 gpurun_out/r04/pytest_lwreg.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/kernel_ab.py --config c3 --stage lw_solver --rounds 9 --iters 20 variants/lw_noreg.so variants/lw_r56.so variants/lw_r48.so variants/lw_r32.so > gpurun_out/r04/lwreg_c3.txt 2>&1 || { tail -5 gpurun_out/r04/lwreg_c3.txt; exit 1; }
grep lw_solver gpurun_out/r04/lwreg_c3.txt
timeout -k 10 300 python -u tools/kernel_ab.py --config c4 --stage lw_solver --rounds 5 --iters 10 variants/lw_noreg.so variants/lw_r56.so variants/lw_r32.so > gpurun_out/r04/lwreg_c4.txt 2>&1 || { tail -5 gpurun_out/r04/lwreg_c4.txt; exit 1; }
grep lw_solver gpurun_out/r04/lwreg_c4.txt
CASES="reg64|default|
noreg|variants/lw_noreg.so|" CONFIGS="c3 c4" REPS=2 STEPS=50 timeout -k 10 600 bash tools/gpu_ab.sh > gpurun_out/r04/lwreg_step.txt 2>&1
rc=$?; cat gpurun_out/r04/lwreg_step.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/kernel_ab.py --config c3 --stage sw_solver --rounds 9 --iters 20 variants/sw_fence.so variants/sw_k4r8.so > gpurun_out/r04/swk3r9_c3.txt 2>&1 || { tail -5 gpurun_out/r04/swk3r9_c3.txt; exit 1; }
grep sw_solver gpurun_out/r04/swk3r9_c3.txt
