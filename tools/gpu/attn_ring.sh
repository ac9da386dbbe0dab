set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 && \
MCP_ATTN_NW4_BUFS=4 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 120 --timeout-method thread >> gpurun_out/attn_tests.log 2>&1 && \
: > gpurun_out/attn_ring.log && \
for q in 16 10 4:16 32; do for b in 2 3 4; do
  MCP_ATTN_NW4_BUFS=$b timeout -k 10 120 python -u tools/bench_attention.py $q | sed "s/^{/{\"nw4_bufs\": $b, /" >> gpurun_out/attn_ring.log || exit 1
done; done
