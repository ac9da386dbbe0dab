set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest4.log 2>&1 || { tail -30 gpurun_out/gputest4.log; exit 1; }
tail -n 1 gpurun_out/gputest4.log
for g in 1 0 1; do
  MCP_NATIVE_GRAMMAR=$g timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 > gpurun_out/gab_$g.log 2>&1 || exit 1
  echo "native_grammar=$g $(grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' gpurun_out/gab_$g.log | tr '\n' ' ') $(grep -o 'schedule_s=[0-9.]*\|update_s=[0-9.]*\|steps=[0-9]*' gpurun_out/gab_$g.log | tr '\n' ' ')"
done
for g in 1 0; do
  MCP_NATIVE_GRAMMAR=$g timeout -k 10 300 python -u bench_serve.py qps --qps 40 --duration 12 > gpurun_out/gq40_$g.json 2> gpurun_out/gq40_$g.err || exit 1
  echo "native_grammar=$g q40 $(grep -o '"p50_latency_ms": [0-9.]*, "p99_latency_ms": [0-9.]*' gpurun_out/gq40_$g.json)"
done
