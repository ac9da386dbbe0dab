set -o pipefail
mkdir -p gpurun_out/gk
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_tp_engine_gpu.py tests/test_engine_splitkv_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gk/tests.log 2>&1 || { tail -30 gpurun_out/gk/tests.log; exit 1; }
tail -1 gpurun_out/gk/tests.log
timeout -k 10 300 python -u bench_serve.py single --n 16 > gpurun_out/gk/single.json 2> gpurun_out/gk/single.err || exit 1
grep -o '"p50_warm_prefix_ms": [0-9.]*, "p90_warm_prefix_ms": [0-9.]*, "p50_cold_prefix_ms": [0-9.]*' gpurun_out/gk/single.json
for q in 40 80 120; do
  timeout -k 10 300 python -u bench_serve.py qps --qps $q --duration 12 > gpurun_out/gk/q$q.json 2> gpurun_out/gk/q$q.err || exit 1
  echo "q=$q $(grep -o '"p50_latency_ms": [0-9.]*, "p99_latency_ms": [0-9.]*' gpurun_out/gk/q$q.json) $(grep -o '"graph_steps": [0-9]*, "steps": [0-9]*, "graph_captures_startup": [0-9]*, "graph_warm_s": [0-9.]*' gpurun_out/gk/q$q.json)"
done
