#!/bin/bash
# Headline A/B: shipped GEMM plan vs a candidate plan file ($2), alternated.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4w}
CAND=${2:?candidate plan path}
mkdir -p $O
for v in ship cand ship cand; do
  if [ $v = cand ]; then export MCP_GEMM_PLAN=$CAND; else unset MCP_GEMM_PLAN; fi
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench_$v.json 2> $O/bench_$v.log || { echo "bench $v failed"; tail -20 $O/bench_$v.log; exit 1; }
  echo "$v $(cut -c1-240 $O/bench_$v.json)" | tee -a $O/ab.txt
done
