#!/bin/bash
# Block-table lane cache in the attention kernels and the prefix pass's 3-deep
# DMA ring: attention / cascade GPU tests, then the attention microbenchmark at
# the headline's shapes (ring 2 / 3 alternated for 16 new tokens and for a
# 2816-key prefix; 8 and 4:16 new tokens at the default).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4g}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention or cascade or prefix or decode or split" > $O/attn_tests.log 2>&1 || { echo "attention tests failed"; tail -30 $O/attn_tests.log; exit 1; }
tail -1 $O/attn_tests.log
for r in 2 3 2 3; do
  MCP_ATTN_PREFIX_RING=$r timeout -k 10 120 python -u tools/bench_attention.py 16 > $O/attn_16_ring$r.log 2>&1 || { echo "bench_attention ring $r failed"; tail -5 $O/attn_16_ring$r.log; exit 1; }
  echo "ql 16 ring $r: $(tail -1 $O/attn_16_ring$r.log)"
done
for r in 2 3; do
  ATTN_PREFIX=2816 MCP_ATTN_PREFIX_RING=$r timeout -k 10 120 python -u tools/bench_attention.py 16 > $O/attn_16_p2816_ring$r.log 2>&1 || { echo "bench_attention 2816 failed"; exit 1; }
  echo "ql 16 prefix 2816 ring $r: $(tail -1 $O/attn_16_p2816_ring$r.log)"
done
for a in 8 4:16; do
  timeout -k 10 120 python -u tools/bench_attention.py $a > $O/attn_$a.log 2>&1 || { echo "bench_attention $a failed"; tail -5 $O/attn_$a.log; exit 1; }
  echo "ql $a: $(tail -1 $O/attn_$a.log)"
done
