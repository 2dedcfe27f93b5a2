#!/bin/bash
# A/B of the fused step's issue order (class-layer order vs FUSED_ORDER), both configs, alternating runs.
set -u
export TMPDIR=/tmp
for cfg in ${CONFIGS:-c3 c4}; do for o in class new class new; do
  RRTMGPNN_STEP_ORDER=$o timeout -k 10 300 python bench.py --config $cfg --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ab_${cfg}_$o.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_${cfg}_$o.json')); print('$cfg $o', d['value'], d['ms_per_step'], d['stages_ms']['sw_solver'], d['stages_overlapped_ms'])"
done; done
