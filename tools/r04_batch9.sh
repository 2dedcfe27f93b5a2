#!/bin/bash
# Round 4, batch 9: the SW checkpoints in one buffer range per column, a ring of 9 levels in the large-grid instances
# and a 3-wave floor for the large clear-sky one -- the SW parity tests (full-size C4 and C5 shard included), each
# config's SW solver alone against the previous build (head.so) and a 2-wave C5 floor, then whole C4 steps.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gpt.py tests/test_gpu_clouds.py tests/test_gpu_fullsize.py tests/test_gpu_fused.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/r04/pytest_b9.log 2>&1
rc=$?; tail -2 gpurun_out/r04/pytest_b9.log; [ $rc -eq 0 ] || exit $rc
for c in c3 c4; do
  timeout -k 10 300 python -u tools/kernel_ab.py --config $c --stage sw_solver --rounds 9 --iters 10 variants/head.so > gpurun_out/r04/swr9_$c.txt 2>&1 || { tail -5 gpurun_out/r04/swr9_$c.txt; exit 1; }
  grep sw_solver gpurun_out/r04/swr9_$c.txt
done
timeout -k 10 600 python -u tools/kernel_ab.py --config c5 --stage sw_solver --rounds 5 --iters 4 variants/head.so variants/nnw2.so > gpurun_out/r04/swr9_c5.txt 2>&1 || { tail -5 gpurun_out/r04/swr9_c5.txt; exit 1; }
grep sw_solver gpurun_out/r04/swr9_c5.txt
CASES="new|default|
head|variants/head.so|" CONFIGS="c4" REPS=3 STEPS=30 timeout -k 10 600 bash tools/gpu_ab.sh > gpurun_out/r04/swr9_step.txt 2>&1
rc=$?; cat gpurun_out/r04/swr9_step.txt; exit $rc
