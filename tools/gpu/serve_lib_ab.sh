set -o pipefail
mkdir -p gpurun_out/slab
for lib in 1 0; do
  export MCP_GEMM_LIB=$lib
  timeout -k 10 300 python -u bench_serve.py single --n 16 > gpurun_out/slab/single_$lib.json 2> gpurun_out/slab/single_$lib.err || exit 1
  for q in 40 80 120; do
    timeout -k 10 300 python -u bench_serve.py qps --qps $q --duration 12 > gpurun_out/slab/q${q}_$lib.json 2> gpurun_out/slab/q${q}_$lib.err || exit 1
    echo "lib=$lib q=$q $(grep -o '"p50_latency_ms": [0-9.]*, "p99_latency_ms": [0-9.]*' gpurun_out/slab/q${q}_$lib.json)"
  done
  echo "lib=$lib single $(grep -o '"p50_latency_ms": [0-9.]*' gpurun_out/slab/single_$lib.json)"
done
