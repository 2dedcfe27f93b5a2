set -u
export TMPDIR=/tmp
for cfg in c3 c4; do for k in 1 2 1 2; do
  timeout -k 10 300 python bench.py --config $cfg --steps 50 --warmup 5 --no-cpu-baseline --sw-kernel $k > gpurun_out/b_${cfg}_$k.json 2> gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/b_${cfg}_$k.json')); print('$cfg sw$k', d['value'], d['ms_per_step'], d['stages_ms']['sw_solver'])"
done; done
