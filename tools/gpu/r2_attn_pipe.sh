set -o pipefail
mkdir -p gpurun_out/ap
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_custom_allreduce_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ap/tests.log 2>&1 || { tail -40 gpurun_out/ap/tests.log; exit 1; }
tail -1 gpurun_out/ap/tests.log
for q in 40 80 120; do
for ps in 0 -1; do
  MCP_PREFIX_SPLIT=$ps timeout -k 10 300 python -u bench_serve.py qps --qps $q --duration 12 > gpurun_out/ap/q${q}_ps$ps.json 2> gpurun_out/ap/q${q}_ps$ps.err || exit 1
  echo "q=$q prefix_split=$ps $(grep -o '"p50_latency_ms": [0-9.]*, "p99_latency_ms": [0-9.]*' gpurun_out/ap/q${q}_ps$ps.json)"
done
done
bash tools/gpu/pipe128.sh
