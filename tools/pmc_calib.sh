#!/bin/bash
# Build tools/pmc_calib.hip on the GPU box and calibrate FETCH_SIZE / WRITE_SIZE (two separate --pmc passes);
# result in gpurun_out/pmc_calib.json.
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
/opt/rocm/bin/hipcc -O3 -shared -fPIC -fno-slp-vectorize --offload-arch=gfx950 tools/pmc_calib.hip -o $TMPDIR/_pmc_calib.so || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 180 rocprofv3 --pmc $c -d gpurun_out/calib_$c -o run --output-format csv -- python3 tools/pmc_calib.py run $TMPDIR/_pmc_calib.so > gpurun_out/calib_$c.log 2>&1 || exit $?
done
python3 tools/pmc_calib.py parse gpurun_out/calib_FETCH_SIZE gpurun_out/calib_WRITE_SIZE gpurun_out/pmc_calib.json || exit $?
# VALU issue: the SQ counters of a pure v_fma_f32 / v_fma_f64 kernel at a known instruction count
timeout -k 10 180 python3 tools/pmc_calib.py valu $TMPDIR/_pmc_calib.so > gpurun_out/calib_valu_times.json || exit $?
cat gpurun_out/calib_valu_times.json
timeout -k 10 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/calib_SQ -o run --output-format csv -- python3 tools/pmc_calib.py valu $TMPDIR/_pmc_calib.so > gpurun_out/calib_SQ.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, json
acc = {}
for f in glob.glob("gpurun_out/calib_SQ/**/*counter_collection*.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0].replace("void ", "")
        acc.setdefault(k, {}).setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
out = {}
for k, d in acc.items():
    r = {c: v[-1] for c, v in d.items()}  # the last dispatch (the timed one)
    if r.get("SQ_BUSY_CYCLES"):
        r["valu_busy"] = 4.0 * r["SQ_ACTIVE_INST_VALU"] / (r["SQ_BUSY_CYCLES"] / 32 * 1024)
    out[k] = r
print(json.dumps(out, indent=1))
json.dump(out, open("gpurun_out/calib_valu_sq.json", "w"), indent=1)
PY
