set -o pipefail
mkdir -p gpurun_out/as
export TMPDIR=/tmp
for S in 4 8 16 32 256; do
for ql in 4 12 4:12; do
for env in "MCP_PREFIX_SPLIT=0 MCP_ATTN_CONCURRENT=0" "MCP_PREFIX_SPLIT=-1 MCP_ATTN_CONCURRENT=0" "MCP_PREFIX_SPLIT=0 MCP_ATTN_CONCURRENT=1" "MCP_CASCADE_OFF=1"; do
  if [ "$env" = "MCP_CASCADE_OFF=1" ]; then continue; fi
  env ATTN_S=$S ATTN_OWN=120 $env timeout -k 10 120 python -u tools/bench_attention.py $ql >> gpurun_out/as/res.jsonl 2>gpurun_out/as/err.txt || { tail -5 gpurun_out/as/err.txt; exit 1; }
  echo "$env" >> gpurun_out/as/res.jsonl
done
done
done
cat gpurun_out/as/res.jsonl
