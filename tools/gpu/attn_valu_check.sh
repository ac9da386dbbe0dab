#!/bin/bash
# Attention VALU trims (fma softmax, prefix pass two tiles per trip): attention
# GPU tests, microbenchmark, headline bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4m}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention or cascade or prefix or decode or split" > $O/attn_tests.log 2>&1 || { echo "attention tests failed"; tail -30 $O/attn_tests.log; exit 1; }
tail -1 $O/attn_tests.log
for a in 16 8 1; do
  timeout -k 10 120 python -u tools/bench_attention.py $a > $O/attn_$a.log 2>&1 || { echo "bench_attention $a failed"; tail -5 $O/attn_$a.log; exit 1; }
  echo "ql $a: $(tail -1 $O/attn_$a.log | cut -c1-200)"
done
ATTN_PREFIX=2816 timeout -k 10 120 python -u tools/bench_attention.py 16 > $O/attn_16_p2816.log 2>&1 || { echo "bench 2816 failed"; exit 1; }
echo "ql 16 prefix 2816: $(tail -1 $O/attn_16_p2816.log | cut -c1-200)"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.log || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
cut -c1-330 $O/bench.json
