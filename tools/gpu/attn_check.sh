set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 && \
: > gpurun_out/attn_check.log && \
for q in 16 10 4; do timeout -k 10 120 python -u tools/bench_attention.py $q >> gpurun_out/attn_check.log 2>&1 || exit 1; done
