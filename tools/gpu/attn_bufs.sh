set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/attn_bufs.log
for b in 2 1 2 1; do
  MCP_ATTN_NW4_BUFS=$b timeout -k 10 120 python -u tools/bench_attention.py 16 | sed "s/^{/{\"nw4_bufs\": $b, /" >> gpurun_out/attn_bufs.log || exit 1
done
for q in 8 32; do for b in 2 1; do
  MCP_ATTN_NW4_BUFS=$b timeout -k 10 120 python -u tools/bench_attention.py $q | sed "s/^{/{\"nw4_bufs\": $b, /" >> gpurun_out/attn_bufs.log || exit 1
done; done
