#!/bin/bash
# Build tools/pmc_calib.hip on the GPU box and calibrate FETCH_SIZE / WRITE_SIZE (two separate --pmc passes);
# result in gpurun_out/pmc_calib.json.
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
/opt/rocm/bin/hipcc -O3 -shared -fPIC --offload-arch=gfx950 tools/pmc_calib.hip -o $TMPDIR/_pmc_calib.so || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 180 rocprofv3 --pmc $c -d gpurun_out/calib_$c -o run --output-format csv -- python3 tools/pmc_calib.py run $TMPDIR/_pmc_calib.so > gpurun_out/calib_$c.log 2>&1 || exit $?
done
python3 tools/pmc_calib.py parse gpurun_out/calib_FETCH_SIZE gpurun_out/calib_WRITE_SIZE gpurun_out/pmc_calib.json
