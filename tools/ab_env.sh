#!/bin/bash
# A/B of a host-side environment knob on the bench line: bash tools/ab_env.sh VAR "v1 v2 ..." (alternating runs, each
# config twice; values may be paths, e.g. RRTMGPNN_LIB builds of tools/solver_variants.sh)
set -u
export TMPDIR=/tmp
VAR=$1; VALS=$2
for cfg in ${CONFIGS:-c3 c4}; do for rep in 1 2; do i=0; for v in $VALS; do i=$((i+1))
  env $VAR=$v timeout -k 10 300 python bench.py --config $cfg --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ab_${cfg}_$i.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_${cfg}_$i.json')); print('$cfg', '$(basename $v)', d['value'], d['ms_per_step'])"
done; done; done
