set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/la_tests.log 2>&1 || { tail -20 gpurun_out/la_tests.log; exit 1; }
tail -n 1 gpurun_out/la_tests.log
for la in 1 0 1 0; do
  MCP_LAUNCH_AHEAD=$la timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 > gpurun_out/la_$la.log 2>&1 || exit 1
  echo "launch_ahead=$la $(grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' gpurun_out/la_$la.log | tr '\n' ' ')"
done
