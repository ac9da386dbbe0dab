#!/bin/bash
# Config 3 end to end at top-32 and top-16 retrieval (block-level prefix
# reuse hit rate reported), and the simulated TP=8 rank of config 4.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4h}
mkdir -p $O
for k in 32 16; do
  MCP_TOPK=$k timeout -k 10 420 python -u bench_suite.py e2e --n 10000 --runs 20 --clients 16 > $O/e2e_top$k.jsonl 2> $O/e2e_top$k.log || { echo "e2e top$k failed"; tail -20 $O/e2e_top$k.log; exit 1; }
  cut -c1-420 $O/e2e_top$k.jsonl
done
timeout -k 10 600 python -u bench_tp.py --simulate-rank 8 --model llama3-70b --steps 2 --warmup 1 > $O/tp8_sim.json 2> $O/tp8_sim.log || { echo "simulate-rank failed"; tail -30 $O/tp8_sim.log; exit 1; }
cat $O/tp8_sim.json
