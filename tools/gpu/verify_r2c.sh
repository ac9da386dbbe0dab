set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest5.log 2>&1 || { tail -30 gpurun_out/gputest5.log; exit 1; }
tail -n 1 gpurun_out/gputest5.log
timeout -k 10 120 python -u tools/bench_swiglu_mid.py 1600 4096 64 > gpurun_out/sw_new.jsonl 2>/dev/null || exit 1
timeout -k 10 300 python -u tools/bench_gemm_mix.py > gpurun_out/gemm_mix2.jsonl 2>/dev/null || exit 1
tail -n 4 gpurun_out/gemm_mix2.jsonl
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_r2c_$i.log 2>&1 || exit 1
  echo "bench $(grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' gpurun_out/bench_r2c_$i.log | tr '\n' ' ')"
done
