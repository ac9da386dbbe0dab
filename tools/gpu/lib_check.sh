set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "library_buckets" -x -q --timeout 120 --timeout-method thread > gpurun_out/lib_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench_lib.log 2>&1 && \
bash tools/gpu/prof_r2b.sh
