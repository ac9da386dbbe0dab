#!/bin/bash
# Config 3 end to end with fixed 5-node plans (top-32), and the simulated TP=8
# rank of config 4 with the TP shard plan.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4t}
mkdir -p $O
timeout -k 10 420 python -u bench_suite.py e2e --n 10000 --runs 20 --clients 16 > $O/e2e.jsonl 2> $O/e2e.log || { echo "e2e failed"; tail -20 $O/e2e.log; exit 1; }
cut -c1-700 $O/e2e.jsonl
timeout -k 10 600 python -u bench_tp.py --simulate-rank 8 --model llama3-70b --steps 2 --warmup 1 > $O/tp8_sim.json 2> $O/tp8_sim.log || { echo "simulate-rank failed"; tail -30 $O/tp8_sim.log; exit 1; }
cat $O/tp8_sim.json
