set -o pipefail
mkdir -p gpurun_out/pc
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_edge_cases_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pc/tests.log 2>&1 || { tail -30 gpurun_out/pc/tests.log; exit 1; }
tail -1 gpurun_out/pc/tests.log
for q in 40 80 120 160; do
  timeout -k 10 300 python -u bench_serve.py qps --qps $q --duration 15 > gpurun_out/pc/qps_$q.json 2> gpurun_out/pc/qps_$q.err || exit 1
  echo "q=$q $(cat gpurun_out/pc/qps_$q.json)"
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/pc/bench.json 2> gpurun_out/pc/bench.err && cat gpurun_out/pc/bench.json
