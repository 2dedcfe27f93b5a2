set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gas_optics or both_model or col_dry or gases or rfmip or fused or probe or fullsize or mlp" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
CASES='new|default|
prev|variants/prev.so|' REPS=2 bash tools/gpu_ab.sh
