set -o pipefail
mkdir -p gpurun_out/configs
timeout -k 10 300 python -u bench_serve.py single > gpurun_out/configs/single.log 2>&1 && \
MCP_GEMM_SPLITK128=0 timeout -k 10 300 python -u bench_serve.py single > gpurun_out/configs/single_nosplit.log 2>&1 && \
timeout -k 10 300 python -u bench_serve.py qps --qps 40 --duration 15 > gpurun_out/configs/qps40.log 2>&1 && \
timeout -k 10 200 python -u bench_suite.py topk > gpurun_out/configs/topk.log 2>&1
