#!/bin/bash
# Full -m gpu suite, then the bitwise default build against the opt-in tolerance build on C3/C4 (alternating runs).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rA > gpurun_out/pytest_all.log 2>&1
rc=$?; grep -E "passed|failed|RMS vs oracle" gpurun_out/pytest_all.log | tail -5
[ $rc -le 1 ] || exit $rc
for cfg in c3 c4; do for rep in 1 2; do for lib in librrtmgpnn librrtmgpnn_fastlibm; do
  RRTMGPNN_LIB=$PWD/rte-rrtmgp-nn_amd/$lib.so timeout -k 10 300 python bench.py --config $cfg --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$cfg $lib', round(d['value']), d['ms_per_step'], d['stages_ms'])"
done; done; done
