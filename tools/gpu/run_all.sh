set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gputests.log; exit 1; }
tail -2 gpurun_out/gputests.log
timeout -k 10 300 python -u bench_serve.py qps --qps 80 --duration 10 > gpurun_out/serve_qps80.json 2> gpurun_out/serve_qps80.err && cat gpurun_out/serve_qps80.json
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json
