set -o pipefail
mkdir -p gpurun_out/conc
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_tp_engine_gpu.py -k "cascade or graph or tp2 or attention" -x -q --timeout 300 --timeout-method thread > gpurun_out/conc/tests.log 2>&1 || { tail -30 gpurun_out/conc/tests.log; exit 1; }
tail -1 gpurun_out/conc/tests.log
for c in 1 0; do
for q in 40 80; do
  MCP_ATTN_CONCURRENT=$c timeout -k 10 300 python -u bench_serve.py qps --qps $q --duration 12 > gpurun_out/conc/q${q}_c$c.json 2> gpurun_out/conc/q${q}_c$c.err || exit 1
  echo "concurrent=$c q=$q $(grep -o '"p50_latency_ms": [0-9.]*, "p99_latency_ms": [0-9.]*' gpurun_out/conc/q${q}_c$c.json)"
done
MCP_ATTN_CONCURRENT=$c timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 > gpurun_out/conc/bench_c$c.json 2> gpurun_out/conc/bench_c$c.err || exit 1
echo "concurrent=$c bench $(grep -o '"value": [0-9.]*' gpurun_out/conc/bench_c$c.json) $(grep -o '"p50_latency_ms": [0-9.]*' gpurun_out/conc/bench_c$c.json)"
done
