#!/bin/bash
# Round 4: the step's schedule tests and smoke() on the last tree.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_chunked.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/r04/pytest_check_final.log 2>&1
rc=$?; tail -2 gpurun_out/r04/pytest_check_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
