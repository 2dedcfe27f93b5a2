#!/bin/bash
# Round 4, batch 14: the LW network on part of the chip (rrtmgpnn_context_set_mlp_max_cus, default 3/4 of the CUs
# when the LW chain follows the SW network) -- the overlap and chunked tests, then whole steps against other caps.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_chunked.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/r04/pytest_b14.log 2>&1
rc=$?; tail -2 gpurun_out/r04/pytest_b14.log; [ $rc -eq 0 ] || exit $rc
CASES="cus192|default|
cus256|default|--lw-net-cus 0
cus160|default|--lw-net-cus 160
cus224|default|--lw-net-cus 224" CONFIGS="c3" REPS=3 STEPS=50 timeout -k 10 600 bash tools/gpu_ab.sh > gpurun_out/r04/lwcus_c3.txt 2>&1
rc=$?; cat gpurun_out/r04/lwcus_c3.txt; [ $rc -eq 0 ] || exit $rc
CASES="cus192|default|
cus256|default|--lw-net-cus 0" CONFIGS="c4" REPS=3 STEPS=30 timeout -k 10 600 bash tools/gpu_ab.sh > gpurun_out/r04/lwcus_c4.txt 2>&1
rc=$?; cat gpurun_out/r04/lwcus_c4.txt; [ $rc -eq 0 ] || exit $rc
CASES="cus192|default|
cus256|default|--lw-net-cus 0" CONFIGS="c5" REPS=2 STEPS=10 timeout -k 10 900 bash tools/gpu_ab.sh > gpurun_out/r04/lwcus_c5.txt 2>&1
rc=$?; cat gpurun_out/r04/lwcus_c5.txt; exit $rc
