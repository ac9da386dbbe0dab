set -o pipefail
for i in 1 2 3; do
  timeout -k 10 400 python -u bench.py > gpurun_out/bw_$i.log 2>&1 || { tail -20 gpurun_out/bw_$i.log; exit 1; }
  echo "run $i $(grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' gpurun_out/bw_$i.log | tr '\n' ' ') $(grep -o 'start-up graph capture.*\|[0-9]* lazy graph captures' gpurun_out/bw_$i.log | tr '\n' ' ')"
done
