set -o pipefail
mkdir -p gpurun_out
for q in 1 4 16; do
  MCP_ATTN_NW1_BUFS=2 timeout -k 10 60 python -u tools/bench_attention.py $q >> gpurun_out/attn_ab.log 2>&1 || exit 1
  MCP_ATTN_NW1_BUFS=1 timeout -k 10 60 python -u tools/bench_attention.py $q >> gpurun_out/attn_ab.log 2>&1 || exit 1
done
