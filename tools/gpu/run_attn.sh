set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "attention" > gpurun_out/attn_tests.log 2>&1 || { tail -40 gpurun_out/attn_tests.log; exit 1; }
tail -3 gpurun_out/attn_tests.log
timeout -k 10 300 python -u tools/bench_attention_splitkv.py > gpurun_out/attn_splitkv.jsonl 2>&1; cat gpurun_out/attn_splitkv.jsonl
MCP_ATTN_SPLIT_BUFS=2 timeout -k 10 300 python -u tools/bench_attention_splitkv.py > gpurun_out/attn_splitkv_buf2.jsonl 2>&1; cat gpurun_out/attn_splitkv_buf2.jsonl
