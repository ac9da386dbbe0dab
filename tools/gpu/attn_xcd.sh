set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/attn_xcd.log
for q in ${QLS:-8 6 2:8 4}; do for x in 0 1 0 1; do
  MCP_ATTN_XCD_ORDER=$x timeout -k 10 120 python -u tools/bench_attention.py $q | sed "s/^{/{\"xcd\": $x, /" >> gpurun_out/attn_xcd.log || exit 1
done; done
