#!/bin/bash
# Round 4, final build, part A: the whole -m gpu suite, smoke(), then the C3 and C4 profile sets
# (tools/profile_configs.sh: kernel traces overlapped and --no-overlap, PMC traffic, SQ and MFMA counters, bench line).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/r04/pytest_final.log 2>&1
rc=$?; tail -2 gpurun_out/r04/pytest_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04/smoke_final.log 2>&1
rc=$?; tail -2 gpurun_out/r04/smoke_final.log; [ $rc -eq 0 ] || exit $rc
CONFIGS="c3 c4" bash tools/profile_configs.sh
