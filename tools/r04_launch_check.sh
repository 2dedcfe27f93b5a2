#!/bin/bash
# Round 4: the driver's N=1 command, `bench.py --gpus 2` self-launched (two ranks sharing the box's GPU, gloo), and
# the CPU allotment the box gives a command (affinity, cgroup quota), for the CPU baseline's thread count.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
{
  echo "nproc $(nproc)"
  python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
  for f in /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpuset.cpus.effective; do [ -r $f ] && echo "$f $(cat $f)"; done
  env | grep -E '^(OMP|MKL|GOMP)_' || true
} > gpurun_out/r04/cpu_allotment.txt
cat gpurun_out/r04/cpu_allotment.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04/bench_n1.json 2> gpurun_out/r04/bench_n1.err || { tail -5 gpurun_out/r04/bench_n1.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r04/bench_n1.json')); print('n1', d['value'], d['ms_per_step'], d['ms_per_step_unsettled'], d['cpu_baseline']['value'], d['cpu_baseline']['spread'])"
timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04/bench_n2.json 2> gpurun_out/r04/bench_n2.err || { tail -5 gpurun_out/r04/bench_n2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r04/bench_n2.json')); print('n2', d['n_gpus'], d['value'], d['gather_ms'], json.dumps(d['gather_check']), json.dumps(d['ranks']))"
