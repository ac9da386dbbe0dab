set -o pipefail
mkdir -p gpurun_out/sab2
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_engine_splitkv_gpu.py tests/test_kernels_gpu.py -k "not topk" -x -q --timeout 300 --timeout-method thread > gpurun_out/sab2/tests.log 2>&1 || { tail -30 gpurun_out/sab2/tests.log; exit 1; }
tail -1 gpurun_out/sab2/tests.log
timeout -k 10 300 python -u bench_serve.py single --n 16 > gpurun_out/sab2/single.json 2> gpurun_out/sab2/single.err || exit 1
cat gpurun_out/sab2/single.json
for q in 20 40 80; do
  timeout -k 10 300 python -u bench_serve.py qps --qps $q --duration 12 > gpurun_out/sab2/q$q.json 2> gpurun_out/sab2/q$q.err || exit 1
  echo "q=$q $(grep -o '"p50_latency_ms": [0-9.]*, "p99_latency_ms": [0-9.]*' gpurun_out/sab2/q$q.json)"
done
