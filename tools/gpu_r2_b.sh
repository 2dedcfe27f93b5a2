#!/bin/bash
# GPU session: new tests, C3 bench (default + tolerance build), C5 global at N=1 (8 chunks), 2-rank gloo rehearsal.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sw_noscat.py tests/test_gpu_tolerance.py tests/test_gpu_glue.py tests/test_gpu_fullsize.py -m gpu -q --timeout 300 --timeout-method thread -rA > gpurun_out/pytest_b.log 2>&1
rc=$?; grep -E "passed|failed|RMS vs oracle" gpurun_out/pytest_b.log | tail -5
[ $rc -le 1 ] || exit $rc
for lib in librrtmgpnn librrtmgpnn_fastlibm; do
  RRTMGPNN_LIB=$PWD/rte-rrtmgp-nn_amd/$lib.so timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/b_$lib.json 2> gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/b_$lib.json')); print('c3 $lib', round(d['value']), d['ms_per_step'], d['stages_ms'])"
done
RRTMGPNN_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b_n2.json 2> gpurun_out/b_n2.err || { tail -5 gpurun_out/b_n2.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/b_n2.json').read().strip().splitlines()[-1]); print('n2', d['value'], d['ms_per_step'], d['gather_ms'], d['end_to_end'], d['config']['global_columns'])"
timeout -k 10 600 python -u bench.py --config c5 --global --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_c5g.json 2> gpurun_out/b_c5g.err || { tail -5 gpurun_out/b_c5g.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b_c5g.json')); print('c5 global', d['value'], d['ms_per_step'], d['scaling'], d['config'])"
