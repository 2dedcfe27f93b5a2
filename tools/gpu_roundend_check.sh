#!/bin/bash
# Round-end rehearsal on one box: the full -m gpu suite, smoke(), and the N-rank bench path with 2 ranks sharing the
# GPU (gloo; the driver's multi-GPU run uses RCCL, one rank per GPU).  Stops at the first failing step.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_all.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
RRTMGPNN_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err || { tail -5 gpurun_out/bench_n2.err; exit 1; }
head -c 600 gpurun_out/bench_n2.json; echo
