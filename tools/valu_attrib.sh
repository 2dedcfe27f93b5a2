#!/bin/bash
# VALU attribution of the two solvers (round 6): SQ instruction counters per launch of the SW solver and the LW solver
# at CONFIG (default c5: the C5 shard), for the shipped library and the attribution builds under variants/
# (tools/build_variant.sh: fastlibm = -DRRTMGPNN_FAST_LIBM=1; exp_hw_all = every solver exp on v_exp_f32; div_hw = the
# correctly rounded division / reciprocal / sqrt sequences as bare v_rcp_f32 / v_sqrt_f32).  Each counter pass is its
# own rocprofv3 run of tools/kernel_ab.py (both stages, 3 launches each).  One JSON per library:
# gpurun_out/valu_<lib>.json {kernel substring: {counter: mean per launch}}.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
cfg=${CONFIG:-c5}
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P3="SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_CVT"
for lib in default ${VARIANTS:-fastlibm exp_hw_all div_hw}; do
  if [ $lib = default ]; then L=$PWD/rte-rrtmgp-nn_amd/librrtmgpnn.so; else L=$PWD/variants/$lib.so; fi
  i=0
  for P in "$P2" "$P3"; do
    i=$((i+1))
    rm -rf gpurun_out/valu_${lib}_$i
    timeout -s KILL 180 rocprofv3 --pmc $P -d gpurun_out/valu_${lib}_$i -o run --output-format csv -- python3 tools/kernel_ab.py --config $cfg --stage sw_solver,lw_solver --base $L --rounds 1 --iters 3 > gpurun_out/valu_${lib}_$i.log 2>&1 || { echo "pmc pass $i of $lib failed"; tail -3 gpurun_out/valu_${lib}_$i.log; exit 1; }
  done
  python3 - "$lib" <<'PY'
import csv, glob, json, sys
lib = sys.argv[1]
acc = {}
for f in glob.glob("gpurun_out/valu_%s_*/**/*counter_collection*.csv" % lib, recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        kern = "sw_solver" if "sw_2stream" in name else ("lw_solver" if "lw_noscat" in name else None)
        if kern is None:
            continue
        d = acc.setdefault(kern, {})
        s, n = d.get(r["Counter_Name"], (0.0, 0))
        d[r["Counter_Name"]] = (s + float(r["Counter_Value"]), n + 1)
res = {k: {c: s / n for c, (s, n) in sorted(v.items())} for k, v in acc.items()}
json.dump(res, open("gpurun_out/valu_%s.json" % lib, "w"), indent=1)
for k, v in sorted(res.items()):
    kc = v.get("SQ_BUSY_CYCLES", 0) / 32
    print(lib, k, "VALU %.3e" % v.get("SQ_INSTS_VALU", 0), "FMA_F64 %.3e" % v.get("SQ_INSTS_VALU_FMA_F64", 0),
          "TRANS_F32 %.3e" % v.get("SQ_INSTS_VALU_TRANS_F32", 0),
          "valu_busy %.3f" % (v.get("SQ_ACTIVE_INST_VALU", 0) * 4 / max(kc * 1024, 1)))
PY
done
