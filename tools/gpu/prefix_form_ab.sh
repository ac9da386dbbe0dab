#!/bin/bash
# Headline: cascade prefix pass forms at the compact view's step sizes
# (default 8 waves x 2 row tiles; 4 waves x 2 (twice the blocks); 4 waves x 4).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4au}
mkdir -p $O
for v in d nw4 rt4 d nw4 rt4; do
  unset MCP_ATTN_PREFIX_NW MCP_ATTN_PREFIX_RT
  if [ $v = nw4 ]; then export MCP_ATTN_PREFIX_NW=4; fi
  if [ $v = rt4 ]; then export MCP_ATTN_PREFIX_RT=4; fi
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench_$v.json 2> $O/bench_$v.log || { echo "bench $v failed"; tail -20 $O/bench_$v.log; exit 1; }
  echo "$v $(cut -c1-300 $O/bench_$v.json)" | tee -a $O/ab.txt
done
