set -o pipefail
mkdir -p gpurun_out/ft
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" > gpurun_out/ft/tests.log 2>&1 || { tail -30 gpurun_out/ft/tests.log; exit 1; }
tail -2 gpurun_out/ft/tests.log
timeout -k 10 600 python -u tools/tune_gemm_plan.py gpurun_out/ft/plan.json > gpurun_out/ft/tune.log 2>&1 || { tail -20 gpurun_out/ft/tune.log; exit 1; }
tail -5 gpurun_out/ft/tune.log | cut -c1-400
