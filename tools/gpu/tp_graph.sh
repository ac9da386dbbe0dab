set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tp_engine_gpu.py tests/test_custom_allreduce_gpu.py tests/test_tp_gpu.py tests/test_engine_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/tp_graph.log 2>&1 || { tail -60 gpurun_out/tp_graph.log; exit 1; }
tail -15 gpurun_out/tp_graph.log
