#!/bin/bash
# SQ / MFMA / LDS counters of the LW MLP for each tiling (RRTMGPNN_MLP32=1: 32x32x2, 0: 16x16x4), one config.
# Each counter set is its own rocprofv3 --pmc run; stops at the first failing step.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
cfg=${CONFIG:-c4}
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
MFMA="SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CYCLES SQ_WAVES"
LDS="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES SQ_WAVES"
for v in ${VALS:-1 0}; do for set in SQ MFMA LDS; do
  o=gpurun_out/mlp_pmc_${cfg}_${v}_$set
  RRTMGPNN_MLP32=$v timeout -s KILL 120 rocprofv3 --pmc ${!set} -d $o -o run --output-format csv -- python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-graph > $o.log 2>&1 || { echo "pmc $v $set failed"; tail -5 $o.log; exit 1; }
  python3 tools/pmc_counters.py $o gpurun_out/mlp_pmc_${cfg}_${v}_$set.json > /dev/null || exit 1
  python3 -c "
import json; r=json.load(open('gpurun_out/mlp_pmc_${cfg}_${v}_$set.json'))
for st in ('predict_nn_lw','predict_nn_sw','sw_solver','lw_solver'):
    if st in r: print('mlp32=$v $set', st, {k: (round(x,4) if isinstance(x,float) else x) for k,x in r[st].items()})
"
done; done
