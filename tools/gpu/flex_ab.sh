set -o pipefail
mkdir -p gpurun_out/fab
export TMPDIR=/tmp
for p in new old; do
  if [ $p = old ]; then export MCP_GEMM_PLAN=tools/gpu/plan_prev.json; else unset MCP_GEMM_PLAN; fi
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 > gpurun_out/fab/bench_$p.json 2> gpurun_out/fab/bench_$p.err || { tail -20 gpurun_out/fab/bench_$p.err; exit 1; }
  echo "$p bench $(grep -o '"value": [0-9.]*' gpurun_out/fab/bench_$p.json)"
  timeout -k 10 300 python -u bench_serve.py single --n 12 > gpurun_out/fab/single_$p.json 2> gpurun_out/fab/single_$p.err || exit 1
  echo "$p single $(grep -o '"p50_warm_prefix_ms": [0-9.]*' gpurun_out/fab/single_$p.json)"
  for q in 40 80 120; do
    timeout -k 10 300 python -u bench_serve.py qps --qps $q --duration 12 > gpurun_out/fab/q${q}_$p.json 2> gpurun_out/fab/q${q}_$p.err || exit 1
    echo "$p q=$q $(grep -o '"p50_latency_ms": [0-9.]*, "p99_latency_ms": [0-9.]*' gpurun_out/fab/q${q}_$p.json)"
  done
done
