set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 200 python -u tools/bench_gemm.py 2048,4096 > gpurun_out/bench_gemm.log 2>&1
