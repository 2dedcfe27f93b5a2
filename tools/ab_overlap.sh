#!/bin/bash
# A/B of the step's two-stream overlap against one stream (alternating runs, both configs)
set -u
export TMPDIR=/tmp
for cfg in ${CONFIGS:-c3 c4}; do for rep in 1 2; do for o in "" "--no-overlap"; do
  timeout -k 10 300 python bench.py --config $cfg --steps 50 --warmup 5 --no-cpu-baseline $o > gpurun_out/abo.json 2> gpurun_out/abo.err || { tail -5 gpurun_out/abo.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/abo.json')); print('$cfg', '${o:-overlap}', d['value'], d['ms_per_step'])"
done; done; done
