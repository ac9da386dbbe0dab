set -o pipefail
mkdir -p gpurun_out/r2m
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2m/gputests.log 2>&1 || { tail -40 gpurun_out/r2m/gputests.log; exit 1; }
tail -2 gpurun_out/r2m/gputests.log
timeout -k 10 300 python -u bench_serve.py single > gpurun_out/r2m/single.json 2> gpurun_out/r2m/single.err || exit 1
cat gpurun_out/r2m/single.json
: > gpurun_out/r2m/qps_sweep.jsonl
for q in 20 40 80 120 160 200; do
  timeout -k 10 300 python -u bench_serve.py qps --qps $q --duration 15 > gpurun_out/r2m/qps_$q.json 2> gpurun_out/r2m/qps_$q.err || exit 1
  cat gpurun_out/r2m/qps_$q.json >> gpurun_out/r2m/qps_sweep.jsonl
done
cat gpurun_out/r2m/qps_sweep.jsonl
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2m/bench.json 2> gpurun_out/r2m/bench.err && cat gpurun_out/r2m/bench.json
