set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -k "full_width" -x -v --timeout 500 --timeout-method thread > gpurun_out/t8b.log 2>&1 || { tail -40 gpurun_out/t8b.log; exit 1; }
tail -3 gpurun_out/t8b.log
