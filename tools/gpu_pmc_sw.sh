#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) and SQ issue counters of the SW solver modes at one config,
# for the default build and variants/<name>.so builds.  gpurun_out/pmc_<cfg>_<lib>_sw<k>_{traffic,sq}.json
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
cfg=${CONFIG:-c3}
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
for lib in default ${VARIANTS:-}; do for k in ${MODES:-2 3}; do
  if [ $lib = default ]; then L=$PWD/rte-rrtmgp-nn_amd/librrtmgpnn.so; else L=$PWD/variants/$lib.so; fi
  tag=${cfg}_${lib}_sw$k
  for c in FETCH_SIZE WRITE_SIZE; do
    RRTMGPNN_LIB=$L timeout -k 10 200 rocprofv3 --pmc $c -d gpurun_out/p_${tag}_$c -o run --output-format csv -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-graph --sw-kernel $k > gpurun_out/p_${tag}_$c.log 2>&1 || { echo "pmc $c failed"; tail -3 gpurun_out/p_${tag}_$c.log; exit 1; }
  done
  python3 tools/pmc_traffic.py gpurun_out/p_${tag}_FETCH_SIZE gpurun_out/p_${tag}_WRITE_SIZE $cfg gpurun_out/pmc_${tag}_traffic.json > /dev/null || exit 1
  RRTMGPNN_LIB=$L timeout -k 10 200 rocprofv3 --pmc $SQ -d gpurun_out/p_${tag}_sq -o run --output-format csv -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-graph --sw-kernel $k > gpurun_out/p_${tag}_sq.log 2>&1 || { echo "pmc sq failed"; exit 1; }
  python3 tools/pmc_counters.py gpurun_out/p_${tag}_sq gpurun_out/pmc_${tag}_sq.json > /dev/null || exit 1
  python3 - $tag <<'PY'
import json, sys
t = json.load(open("gpurun_out/pmc_%s_traffic.json" % sys.argv[1]))
q = json.load(open("gpurun_out/pmc_%s_sq.json" % sys.argv[1]))
x = t.get("sw_solver", t); y = q.get("sw_solver", {})
print(sys.argv[1], "traffic", json.dumps(x)[:300])
print(sys.argv[1], "sq", {k: y.get(k) for k in ("frac_wait_any", "frac_wait_inst_any", "frac_active_inst_valu", "valu_insts_per_wave", "SQ_WAVES")})
PY
done; done
