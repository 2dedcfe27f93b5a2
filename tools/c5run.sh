set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/c5
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || echo "list rc=$?"
grep -i "mfma" gpurun_out/counters_list.txt | head -40
timeout -k 10 400 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/c5/bench.json 2> gpurun_out/c5/bench.err
rc=$?; echo "c5 rc=$rc"; cat gpurun_out/c5/bench.json; tail -5 gpurun_out/c5/bench.err
exit $rc
