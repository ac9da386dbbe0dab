set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_engine_splitkv_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/graph_tests.log 2>&1 || { tail -40 gpurun_out/graph_tests.log; exit 1; }
tail -3 gpurun_out/graph_tests.log
for q in 40 80 160; do
timeout -k 10 200 python -u bench_serve.py qps --qps $q --duration 10 > gpurun_out/serve_q$q.json 2> gpurun_out/serve_q$q.err || exit 1
cat gpurun_out/serve_q$q.json
done
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json
