#!/bin/bash
# Round 4, final build, part B: the C5 shard profile set, the driver's bench command (with the CPU baseline), and
# `python bench.py --gpus 2` starting its two ranks itself (sharing the one GPU, gloo gather).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
STEPS=10 CONFIGS="c5" bash tools/profile_configs.sh || exit $?
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04/bench_driver_final.json 2> gpurun_out/r04/bench_driver_final.err
rc=$?; head -c 400 gpurun_out/r04/bench_driver_final.json; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04/bench_n2_final.json 2> gpurun_out/r04/bench_n2_final.err
rc=$?; head -c 400 gpurun_out/r04/bench_n2_final.json; echo; exit $rc
