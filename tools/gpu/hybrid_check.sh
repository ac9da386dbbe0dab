set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/hy_tests.log 2>&1 && \
: > gpurun_out/hybrid_ab.log && \
for h in 1 0 1 0; do
  MCP_GEMM_HYBRID=$h timeout -k 10 300 python -u tools/bench_gemm_variants.py 49 "3000,28672,4096;4352,4096,4096;2304,6144,4096;3000,4096,14336;3500,28672,4096;2816,6144,4096" | sed "s/^{/{\"hybrid\": $h, /" >> gpurun_out/hybrid_ab.log || exit 1
done
