set -o pipefail
for t in 4096 3328 4608 5120 4096; do
  timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --max-step-tokens $t > gpurun_out/mst_$t.log 2>&1 || exit 1
  echo "mst=$t $(grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' gpurun_out/mst_$t.log | tr '\n' ' ')"
done
