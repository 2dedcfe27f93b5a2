#!/bin/bash
# Whole-step A/B on one box: for each config and repetition, every case "label|lib|bench args" in CASES (newline
# separated; lib is a path relative to the repo or "default"), alternating.  One line per run.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-50}
for cfg in ${CONFIGS:-c3 c4}; do for rep in $(seq ${REPS:-2}); do
  while IFS='|' read -r label lib args; do
    [ -z "$label" ] && continue
    if [ "$lib" = default ]; then L=$PWD/rte-rrtmgp-nn_amd/librrtmgpnn.so; else L=$PWD/$lib; fi
    RRTMGPNN_LIB=$L timeout -k 10 300 python bench.py --config $cfg --steps $STEPS --warmup 5 --no-cpu-baseline --c5-steps 0 $args > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$cfg', '$label', round(d['value']), d['ms_per_step'], json.dumps(d['stages_ms']), (d['stages_overlapped_ms'] or {}).get('sw_solver'))"
  done <<< "$CASES"
done; done
