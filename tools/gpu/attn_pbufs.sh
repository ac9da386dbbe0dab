set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/attn_pbufs.log
for q in 16 10 4; do for b in 2 1; do
  MCP_ATTN_PREFIX_BUFS=$b timeout -k 10 120 python -u tools/bench_attention.py $q | sed "s/^{/{\"prefix_bufs\": $b, /" >> gpurun_out/attn_pbufs.log || exit 1
done; done
