#!/bin/bash
# Bench lines with the compiled CPU baseline (oracle/_ref/rrtmgp_cpu_bench): C3 twice (run-to-run spread), C1, C4.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in c3 c3 c1 c4; do
  timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 5 --c5-steps 0 > gpurun_out/cpub_$c.json 2> gpurun_out/cpub_$c.err || { tail -5 gpurun_out/cpub_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/cpub_$c.json')); print('$c', d['value'], d['ms_per_step'], json.dumps(d['cpu_baseline']))"
done
