#!/bin/bash
# SQ counters and HBM-side traffic of one stage run alone (tools/kernel_ab.py --stage), for the in-tree library and
# variants/<name>.so builds: passes of at most 8 SQ counters, FETCH_SIZE and WRITE_SIZE in passes of their own.
# CONFIG (c3), STAGE (sw_solver), VARIANTS.  Prints one summary line per library; gpurun_out/stagepmc_<stage>_<lib>.json
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
cfg=${CONFIG:-c3}; stage=${STAGE:-sw_solver}
case $stage in
  sw_solver) kf="sw_2stream" ;; lw_solver) kf="lw_noscat" ;; predict_nn_lw) kf="mlp32_kernel<9" ;;
  predict_nn_sw) kf="mlp32_kernel<4" ;; *) kf=$stage ;;
esac
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VMEM"
P3="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_FMA_F32 SQ_VALU_MFMA_COEXEC_CYCLES"
for lib in default ${VARIANTS:-}; do
  if [ $lib = default ]; then L=$PWD/rte-rrtmgp-nn_amd/librrtmgpnn.so; else L=$PWD/variants/$lib.so; fi
  i=0
  for P in "$P1" "$P2" "$P3" FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/stagepmc_${lib}_$i -o run --output-format csv -- python3 tools/kernel_ab.py --config $cfg --stage $stage --base $L --rounds 1 --iters 3 > gpurun_out/stagepmc_${lib}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 gpurun_out/stagepmc_${lib}_$i.log; exit 1; }
  done
  python3 - "$lib" "$kf" "$stage" <<'PY'
import csv, glob, json, sys
lib, kf, stage = sys.argv[1:4]
acc = {}
for f in glob.glob("gpurun_out/stagepmc_%s_*/**/*counter_collection*.csv" % lib, recursive=True):
    for r in csv.DictReader(open(f)):
        if kf not in r.get("Kernel_Name", ""):
            continue
        k = r["Counter_Name"]
        s, n = acc.get(k, (0.0, 0))
        acc[k] = (s + float(r["Counter_Value"]), n + 1)
res = {k: s / n for k, (s, n) in sorted(acc.items())}
json.dump(res, open("gpurun_out/stagepmc_%s_%s.json" % (stage, lib), "w"), indent=1)
wc = res.get("SQ_WAVE_CYCLES", 1)
kc = res.get("SQ_BUSY_CYCLES", 0) / 32
print(lib, stage, "kernel cycles %.0f" % kc, "valu_busy %.3f" % (res.get("SQ_ACTIVE_INST_VALU", 0) * 4 / max(kc * 1024, 1)),
      "mfma_busy %.3f" % (res.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(kc * 1024, 1)),
      "fetch %.1f MB (x2 for gfx950)" % (res.get("FETCH_SIZE", 0) / 1024), "write %.1f MB" % (res.get("WRITE_SIZE", 0) / 1024))
print(lib, stage, " ".join("%s=%.4g" % (k[3:] if k.startswith("SQ_") else k, v) for k, v in res.items()))
print(lib, stage, "per wave-cycle:", " ".join("%s=%.3f" % (k[3:], res[k] / wc) for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM") if k in res))
PY
done
