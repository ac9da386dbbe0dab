set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tp_engine_gpu.py tests/test_custom_allreduce_gpu.py tests/test_rccl_gpu.py -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/tp_tests.log 2>&1; rc=$?; tail -30 gpurun_out/tp_tests.log; exit $rc
