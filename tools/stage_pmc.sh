#!/bin/bash
# SQ counters of one stage (kernel_ab.py, the stage alone) for the in-tree library and variants/<name>.so builds, in
# passes of at most 8 SQ counters: gpurun_out/swpmc_<lib>.json.  CONFIG (c3), STAGE (sw_solver), VARIANTS.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
cfg=${CONFIG:-c3}; stage=${STAGE:-sw_solver}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM"
P3="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_THREAD_CYCLES_VALU"
P4="SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM_RD SQ_LEVEL_WAVES"
for lib in default ${VARIANTS:-}; do
  if [ $lib = default ]; then L=$PWD/rte-rrtmgp-nn_amd/librrtmgpnn.so; else L=$PWD/variants/$lib.so; fi
  i=0
  for P in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/swpmc_${lib}_$i -o run --output-format csv -- python3 tools/kernel_ab.py --config $cfg --stage $stage --base $L --rounds 1 --iters 3 > gpurun_out/swpmc_${lib}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 gpurun_out/swpmc_${lib}_$i.log; exit 1; }
  done
  python3 - $lib <<'PY'
import csv, glob, json, sys
lib = sys.argv[1]
acc = {}
for f in glob.glob("gpurun_out/swpmc_%s_*/**/*counter_collection*.csv" % lib, recursive=True):
    for r in csv.DictReader(open(f)):
        if "sw_2stream" not in r.get("Kernel_Name", "") and "lw_noscat" not in r.get("Kernel_Name", "") and "mlp" not in r.get("Kernel_Name", ""):
            continue
        k = r["Counter_Name"]
        s, n = acc.get(k, (0.0, 0))
        acc[k] = (s + float(r["Counter_Value"]), n + 1)
res = {k: s / n for k, (s, n) in sorted(acc.items())}
json.dump(res, open("gpurun_out/swpmc_%s.json" % lib, "w"), indent=1)
wc = res.get("SQ_WAVE_CYCLES", 1)
kc = res.get("SQ_BUSY_CYCLES", 0) / 32
print(lib, "kernel_us %.1f" % (kc / 2.4e3), " ".join("%s=%.3g" % (k[3:], v) for k, v in res.items()))
print(lib, "per wave-cycle:", " ".join("%s=%.3f" % (k[3:], res[k] / wc) for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA") if k in res))
PY
done
