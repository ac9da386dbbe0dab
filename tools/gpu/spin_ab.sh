set -o pipefail
for sw in 1 0 1 0; do
  MCP_SPIN_WAIT=$sw timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 > gpurun_out/spin_$sw.log 2>&1 || exit 1
  echo "spin=$sw $(grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' gpurun_out/spin_$sw.log | tr '\n' ' ')"
done
for sw in 1 0; do
  MCP_SPIN_WAIT=$sw timeout -k 10 300 python -u bench_serve.py qps --qps 40 --duration 12 > gpurun_out/spq_$sw.json 2>/dev/null || exit 1
  echo "spin=$sw q40 $(grep -o '"p50_latency_ms": [0-9.]*, "p99_latency_ms": [0-9.]*' gpurun_out/spq_$sw.json)"
done
