#!/bin/bash
# Plan with the same-box codes / splits / flex of the fsplit tunes (M <= 1024,
# 8B + 70B TP=1) vs the shipped plan: config 5 at 120/s, config 4, headline.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4bh}
mkdir -p $O
CAND=${2:?candidate plan path}
for v in ship cand ship cand; do
  if [ $v = cand ]; then export MCP_GEMM_PLAN=$CAND; else unset MCP_GEMM_PLAN; fi
  timeout -k 10 300 python -u bench_serve.py qps --qps 120 --duration 20 > $O/q120_$v.json 2> $O/q120_$v.log || { echo "qps $v failed"; tail -20 $O/q120_$v.log; exit 1; }
  echo "q120 $v $(cut -c1-330 $O/q120_$v.json)" | tee -a $O/ab.txt
  timeout -k 10 500 python -u bench_tp.py --gpus 1 > $O/c4_$v.json 2> $O/c4_$v.log || { echo "config 4 $v failed"; tail -20 $O/c4_$v.log; exit 1; }
  echo "c4 $v $(cut -c1-300 $O/c4_$v.json)" | tee -a $O/ab.txt
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench_$v.json 2> $O/bench_$v.log || { echo "bench $v failed"; tail -20 $O/bench_$v.log; exit 1; }
  echo "head $v $(cut -c1-240 $O/bench_$v.json)" | tee -a $O/ab.txt
done
