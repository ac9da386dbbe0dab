set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_sharded_retrieval_cpu.py -k "topk or retrieval or shard" -x -v --timeout 120 --timeout-method thread > gpurun_out/topk_tests.log 2>&1 || { tail -40 gpurun_out/topk_tests.log; exit 1; }
tail -2 gpurun_out/topk_tests.log
timeout -k 10 300 python -u bench_suite.py topk --n 10000 > gpurun_out/topk_10k.jsonl 2>&1 && cat gpurun_out/topk_10k.jsonl
timeout -k 10 300 python -u bench_suite.py topk --n 10000000 > gpurun_out/topk_10m.jsonl 2>&1 && cat gpurun_out/topk_10m.jsonl
