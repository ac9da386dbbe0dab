set -o pipefail
mkdir -p gpurun_out/nw4
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/nw4/tests0.log 2>&1 || { tail -20 gpurun_out/nw4/tests0.log; exit 1; }
MCP_ATTN_NW4_FORM=1 timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/nw4/tests1.log 2>&1 || { tail -20 gpurun_out/nw4/tests1.log; exit 1; }
tail -1 gpurun_out/nw4/tests0.log gpurun_out/nw4/tests1.log
for ql in 16 10 8 6:12 32; do
  for f in 0 1 0 1; do
    echo "form=$f ql=$ql $(MCP_ATTN_NW4_FORM=$f timeout -k 10 60 python -u tools/bench_attention.py $ql 2>/dev/null | tail -1)"
  done
done
for f in 1 0 1; do
  MCP_ATTN_NW4_FORM=$f timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 > gpurun_out/nw4/bench_$f.log 2>&1 || exit 1
  echo "bench form=$f $(grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' gpurun_out/nw4/bench_$f.log | tr '\n' ' ')"
done
