#!/bin/bash
# A/B of the whole bench between this tree and another checkout built beside it (OLD=path, default build/old),
# alternating runs on one box (box-to-box clock differences exceed the changes being compared).
set -u
export TMPDIR=/tmp
OLD=${OLD:-build/old}
for cfg in ${CONFIGS:-c3 c4}; do for rep in $(seq ${REPS:-3}); do for t in "$OLD" "."; do
  X=""; grep -q -- "--c5-steps" $t/bench.py && X="--c5-steps 0"  # trees before round 5 have no c5_global block
  (cd $t && timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-50} --warmup 5 --no-cpu-baseline $X > /tmp/abt.json 2> /tmp/abt.err) || { tail -5 /tmp/abt.err; exit 1; }
  python3 -c "import json; d=json.load(open('/tmp/abt.json')); print('$cfg', '$t', d['value'], d['ms_per_step'])"
done; done; done
