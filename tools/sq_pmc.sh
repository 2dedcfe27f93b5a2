#!/bin/bash
# SQ stall counters of every stage for each variant build of tools/solver_variants.sh (same "name:flags" specs),
# on one config: rocprofv3 --pmc of the SQ wave/wait/VALU counters, summarised by tools/pmc_counters.py into
# gpurun_out/sq_<config>_<name>.json.  Stops at the first failing GPU step.
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
cfg=${CONFIG:-c3}
bcfg=${BENCH_CONFIG:-$cfg}  # bench.py config of the profiled runs (c4 for the c4a variants)
timeout -k 10 400 bash tools/solver_variants.sh "$@" > gpurun_out/sq_var_$cfg.txt 2>&1 || exit $?
cat gpurun_out/sq_var_$cfg.txt
B=$TMPDIR/rrtmgpnn_var
CTRS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
for spec in "$@"; do
  n=${spec%%:*}
  o=gpurun_out/sq_${cfg}_$n
  RRTMGPNN_LIB=$B/lib_$n.so timeout -k 10 300 rocprofv3 --pmc $CTRS -d $o -o run --output-format csv -- python3 bench.py --config $bcfg --steps 5 --warmup 2 --no-cpu-baseline --no-graph > $o.log 2>&1 || exit $?
  python3 tools/pmc_counters.py $o gpurun_out/sq_${cfg}_$n.json > /dev/null || exit $?
  python3 - "$n" gpurun_out/sq_${cfg}_$n.json <<'PY'
import json, sys
r = json.load(open(sys.argv[2]))
for st in ("sw_solver", "lw_solver", "predict_nn_lw", "predict_nn_sw"):
    if st in r:
        x = r[st]
        print("%-8s %-14s waves %8.0f wait %.3f inst %.3f active %.3f valu %.3f valu/wave %s" % (
            sys.argv[1], st, x.get("SQ_WAVES", 0), x.get("frac_wait_any", 0), x.get("frac_wait_inst_any", 0),
            x.get("frac_active_inst_any", 0), x.get("frac_active_inst_valu", 0), x.get("valu_insts_per_wave")))
PY
done
exit 0
