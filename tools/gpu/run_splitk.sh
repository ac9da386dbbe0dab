set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "splitk" > gpurun_out/splitk_tests.log 2>&1 || { tail -40 gpurun_out/splitk_tests.log; exit 1; }
tail -3 gpurun_out/splitk_tests.log
timeout -k 10 600 python -u tools/bench_splitk.py > gpurun_out/splitk_sweep.jsonl 2>&1
