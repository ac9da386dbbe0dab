set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 && \
timeout -k 10 120 python -u tools/bench_attention.py 16 > gpurun_out/attn_rg.log 2>&1 && \
timeout -k 10 120 python -u tools/bench_attention.py 4 >> gpurun_out/attn_rg.log 2>&1
