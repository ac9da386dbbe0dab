set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/attn_cutoff.log
for q in 10 12 16 4:16; do
  for cfg in "8 0" "16 0" "16 1"; do set -- $cfg
    MCP_ATTN_NW1_CUTOFF=$1 MCP_ATTN_XCD_ORDER=$2 timeout -k 10 120 python -u tools/bench_attention.py $q | sed "s/^{/{\"cutoff\": $1, \"xcd\": $2, /" >> gpurun_out/attn_cutoff.log || exit 1
  done
done
