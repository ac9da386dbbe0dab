set -o pipefail
timeout -k 10 120 python -u tools/bench_swiglu_mid.py 1600 4096 64 > gpurun_out/sw_def.jsonl 2>/dev/null || exit 1
MCP_GEMM_HYBRID=0 timeout -k 10 120 python -u tools/bench_swiglu_mid.py 1600 4096 64 > gpurun_out/sw_h0.jsonl 2>/dev/null || exit 1
MCP_GEMM_TAIL_SPLIT=2 timeout -k 10 120 python -u tools/bench_swiglu_mid.py 1600 4096 64 > gpurun_out/sw_t2.jsonl 2>/dev/null || exit 1
MCP_GEMM_TAIL_SPLIT=8 timeout -k 10 120 python -u tools/bench_swiglu_mid.py 1600 4096 64 > gpurun_out/sw_t8.jsonl 2>/dev/null || exit 1
MCP_GEMM_BM=192 timeout -k 10 120 python -u tools/bench_swiglu_mid.py 1600 4096 64 > gpurun_out/sw_b192.jsonl 2>/dev/null || exit 1
MCP_GEMM_BM=256 timeout -k 10 120 python -u tools/bench_swiglu_mid.py 1600 4096 64 > gpurun_out/sw_b256.jsonl 2>/dev/null || exit 1
