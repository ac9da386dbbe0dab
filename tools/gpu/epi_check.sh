set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/epi_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_gemm_variants.py 49,61,51 "4096,28672,4096;4096,4096,14336;4096,6144,4096;4096,4096,4096;2600,4096,4096;2600,28672,4096;2600,4096,14336;2600,6144,4096" > gpurun_out/epi_ab.log 2>&1 && \
timeout -k 10 200 python -u tools/bench_gemm.py 2600,4096 > gpurun_out/epi_bench_gemm.log 2>&1
