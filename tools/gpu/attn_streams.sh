set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/attn_streams.log
for q in 4:16 2:12 8:24 16; do for st in 1 2 1 2; do
  MCP_ATTN_STREAMS=$st timeout -k 10 120 python -u tools/bench_attention.py $q | sed "s/^{/{\"streams\": $st, /" >> gpurun_out/attn_streams.log || exit 1
done; done
