set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "topk" -x -v --timeout 120 --timeout-method thread > gpurun_out/topk_tests.log 2>&1 || { tail -40 gpurun_out/topk_tests.log; exit 1; }
tail -2 gpurun_out/topk_tests.log
timeout -k 10 300 python -u bench_suite.py topk --n 10000000 > gpurun_out/topk_dsplit.jsonl 2>&1 && cat gpurun_out/topk_dsplit.jsonl
MCP_TOPK_DSPLIT=0 timeout -k 10 300 python -u bench_suite.py topk --n 10000000 > gpurun_out/topk_reg.jsonl 2>&1 && cat gpurun_out/topk_reg.jsonl
