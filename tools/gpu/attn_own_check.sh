#!/bin/bash
# Decode kernel in own-span mode for unsplit steps: GPU tests, then the
# attention microbenchmark (full entry point) with MCP_ATTN_DECODE_OWN 0 / 1 / 2
# at 8 (1-wave items), 16 (4-wave items) and 4:16 new tokens per request.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4i}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "own_span or cascade_fold or paged_attention" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for a in 8 16 4:16 1; do
  for m in 0 1 2 0 1 2; do
    MCP_ATTN_DECODE_OWN=$m timeout -k 10 120 python -u tools/bench_attention.py $a > $O/attn_${a}_m$m.log 2>&1 || { echo "bench $a m$m failed"; tail -5 $O/attn_${a}_m$m.log; exit 1; }
    echo "ql $a own-mode $m: $(tail -1 $O/attn_${a}_m$m.log | cut -c1-160)"
  done
done
