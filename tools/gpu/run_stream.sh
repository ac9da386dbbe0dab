set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "stream or qkv_rope" > gpurun_out/stream_tests.log 2>&1 || { tail -40 gpurun_out/stream_tests.log; exit 1; }
tail -3 gpurun_out/stream_tests.log
timeout -k 10 300 python -u tools/bench_stream.py > gpurun_out/stream3.jsonl 2>&1
