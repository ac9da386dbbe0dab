set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "topk" > gpurun_out/topk_tests.log 2>&1 || { tail -40 gpurun_out/topk_tests.log; exit 1; }
tail -3 gpurun_out/topk_tests.log
timeout -k 10 300 python -u bench_suite.py topk --n 10000 > gpurun_out/topk_10k.jsonl 2>&1; cat gpurun_out/topk_10k.jsonl
timeout -k 10 300 python -u bench_suite.py topk --n 10000000 > gpurun_out/topk_10m.jsonl 2>&1; cat gpurun_out/topk_10m.jsonl
