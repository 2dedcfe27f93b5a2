#!/bin/bash
# A/B the whole step: build the variants of tools/solver_variants.sh ("name:flags" specs) and run bench.py on each
# config (CONFIGS, default "c3 c4") with each variant library in turn, REPS rounds interleaved, printing ms_per_step.
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
BUILD_ONLY=1 bash tools/solver_variants.sh "$@" || exit $?
B=$TMPDIR/rrtmgpnn_var
for rep in $(seq ${REPS:-2}); do
  for cfg in ${CONFIGS:-c3 c4}; do
    for spec in "$@"; do
      n=${spec%%:*}
      RRTMGPNN_LIB=$B/lib_$n.so timeout -k 10 300 python3 bench.py --config $cfg --steps ${STEPS:-50} --warmup 5 --no-cpu-baseline > gpurun_out/ab_${cfg}_$n.json 2> gpurun_out/ab_err.txt || exit $?
      python3 -c "import json,sys; b=json.load(open(sys.argv[1])); print('%s %-3s %-8s %.4f ms/step  sw %.4f' % (sys.argv[2], sys.argv[3], sys.argv[4], b['ms_per_step'], b['stages_ms']['sw_solver']))" gpurun_out/ab_${cfg}_$n.json $rep $cfg $n
    done
  done
done
