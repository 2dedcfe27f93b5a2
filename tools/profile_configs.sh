#!/bin/bash
# Bench + rocprofv3 kernel-trace summary + PMC HBM traffic + SQ issue counters for each config given (default: c3 c4),
# one GPU box call.  Each config's artefacts land in gpurun_out/<config>/; PMC traffic is merged into
# gpurun_out/pmc_traffic.json, the SQ counters (valu_busy etc.) into gpurun_out/pmc_sq.json.
# Stops at the first failing GPU step (every step has its own time limit).
# The kernel trace runs the bench line's own command (LW and SW chains overlapped, as bench.py times its stages),
# so its per-kernel averages are comparable with the line's roofline; a second trace with --no-overlap gives each
# kernel's time with the chip to itself (prof_iso).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-30}
MFMA="SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CYCLES SQ_WAVES"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
for cfg in ${CONFIGS:-c3 c4}; do
  o=gpurun_out/$cfg
  mkdir -p $o
  echo "== $cfg rocprofv3 kernel trace"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run --output-format csv -- python3 bench.py --config $cfg --steps $STEPS --warmup 5 --no-cpu-baseline --c5-steps 0 ${BENCH_ARGS:-} > $o/prof.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof_iso -o run --output-format csv -- python3 bench.py --config $cfg --steps $STEPS --warmup 5 --no-cpu-baseline --c5-steps 0 --no-overlap ${BENCH_ARGS:-} > $o/prof_iso.log 2>&1 || exit $?
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "== $cfg rocprofv3 --pmc $c"
    timeout -k 10 300 rocprofv3 --pmc $c -d $o/pmc_$c -o run --output-format csv -- python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --c5-steps 0 --no-graph --settle-s 0 ${BENCH_ARGS:-} > $o/pmc_$c.log 2>&1 || exit $?
  done
  python3 tools/pmc_traffic.py $o/pmc_FETCH_SIZE $o/pmc_WRITE_SIZE $cfg gpurun_out/pmc_traffic.json > $o/pmc_traffic.txt || exit $?
  echo "== $cfg rocprofv3 --pmc SQ counters"
  timeout -k 10 300 rocprofv3 --pmc $SQ -d $o/pmc_SQ -o run --output-format csv -- python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --c5-steps 0 --no-graph --settle-s 0 ${BENCH_ARGS:-} > $o/pmc_SQ.log 2>&1 || exit $?
  python3 tools/pmc_counters.py $o/pmc_SQ gpurun_out/pmc_sq.json $cfg > $o/pmc_sq.txt || exit $?
  echo "== $cfg rocprofv3 --pmc MFMA counters"
  timeout -k 10 300 rocprofv3 --pmc $MFMA -d $o/pmc_MFMA -o run --output-format csv -- python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --c5-steps 0 --no-graph --settle-s 0 ${BENCH_ARGS:-} > $o/pmc_MFMA.log 2>&1 || exit $?
  python3 tools/pmc_counters.py $o/pmc_MFMA gpurun_out/pmc_sq.json $cfg > $o/pmc_mfma.txt || exit $?
  # the bench line last, so its roofline carries this build's PMC traffic and SQ figures
  echo "== $cfg bench"
  timeout -k 10 300 python bench.py --config $cfg --steps $STEPS --warmup 5 --traffic-json gpurun_out/pmc_traffic.json --sq-json gpurun_out/pmc_sq.json ${BENCH_ARGS:-} > $o/bench.json 2> $o/bench.err || exit $?
  head -c 400 $o/bench.json; echo
done
exit 0
