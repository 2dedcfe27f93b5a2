#!/bin/bash
# Round 4 SW-solver experiment 1: the checkpointed kernel alone (tools/kernel_ab.py, alternating, outputs compared
# bitwise with the default build) against variants/*.so, at C3 and C4; then the whole -m gpu suite on the default build.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
V="variants/nopk.so variants/nofence.so variants/k3.so variants/w3.so variants/p1.so variants/p12.so variants/noflush.so"
timeout -k 10 300 python -u tools/kernel_ab.py --config c3 --stage sw_solver --rounds 9 --iters 20 $V > gpurun_out/r04/swexp1_c3.txt 2>&1 || { tail -5 gpurun_out/r04/swexp1_c3.txt; exit 1; }
cat gpurun_out/r04/swexp1_c3.txt
timeout -k 10 300 python -u tools/kernel_ab.py --config c4 --stage sw_solver --rounds 5 --iters 10 variants/nopk.so variants/nofence.so > gpurun_out/r04/swexp1_c4.txt 2>&1 || { tail -5 gpurun_out/r04/swexp1_c4.txt; exit 1; }
cat gpurun_out/r04/swexp1_c4.txt
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/r04/pytest_gpu_pruned.log 2>&1
rc=$?; tail -4 gpurun_out/r04/pytest_gpu_pruned.log; exit $rc
