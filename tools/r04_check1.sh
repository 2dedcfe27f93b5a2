#!/bin/bash
# Round 4, first GPU call: the g-point / Fortran tests changed this round, then the launch check (bench N=1, N=2).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests/test_gpu_gpt.py tests/test_fortran.py -x -q --timeout 240 --timeout-method thread -rf > gpurun_out/r04/pytest_changed.log 2>&1
rc=$?; tail -4 gpurun_out/r04/pytest_changed.log; [ $rc -eq 0 ] || exit $rc
bash tools/r04_launch_check.sh
