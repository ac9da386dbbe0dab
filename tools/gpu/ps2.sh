set -o pipefail
mkdir -p gpurun_out/ps2
export TMPDIR=/tmp
for ps in -1 0; do
  MCP_PREFIX_SPLIT=$ps timeout -k 10 300 python -u bench_serve.py single --n 12 > gpurun_out/ps2/single_$ps.json 2> gpurun_out/ps2/single_$ps.err || exit 1
  echo "ps=$ps single $(grep -o '"p50_warm_prefix_ms": [0-9.]*' gpurun_out/ps2/single_$ps.json)"
  for q in 20 40 80; do
    MCP_PREFIX_SPLIT=$ps timeout -k 10 300 python -u bench_serve.py qps --qps $q --duration 12 > gpurun_out/ps2/q${q}_$ps.json 2> gpurun_out/ps2/q${q}_$ps.err || exit 1
    echo "ps=$ps q=$q $(grep -o '"p50_latency_ms": [0-9.]*, "p99_latency_ms": [0-9.]*' gpurun_out/ps2/q${q}_$ps.json)"
  done
done
