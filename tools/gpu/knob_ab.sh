set -o pipefail
for kv in "NONE=1" "MCP_ATTN_PREFIX_NW=4" "MCP_ATTN_NW1_BUFS=2" "MCP_GEMM_SK_SMALL=0" "MCP_ATTN_PREFIX_HEAD_MAJOR=0" "NONE=2"; do
  env $kv timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 > gpurun_out/knob.log 2>&1 || exit 1
  echo "$kv $(grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' gpurun_out/knob.log | tr '\n' ' ')"
done
