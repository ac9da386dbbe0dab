#!/bin/bash
# BASELINE configs at HEAD: 2 (single intent), 5 (80 / 120 intents/s),
# 4 (70B TP=1, fixed 5-node plans), 3 (e2e, 10k registry, 16 clients).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4s}
mkdir -p $O
timeout -k 10 300 python -u bench_serve.py single --n 20 > $O/config2.json 2> $O/config2.log || { echo "config 2 failed"; tail -20 $O/config2.log; exit 1; }
cut -c1-400 $O/config2.json
for q in 80 120; do
  timeout -k 10 300 python -u bench_serve.py qps --qps $q --duration 20 > $O/config5_q$q.json 2> $O/config5_q$q.log || { echo "config 5 q$q failed"; tail -20 $O/config5_q$q.log; exit 1; }
  cut -c1-400 $O/config5_q$q.json
done
timeout -k 10 500 python -u bench_tp.py --gpus 1 > $O/config4_tp1.json 2> $O/config4_tp1.log || { echo "config 4 failed"; tail -20 $O/config4_tp1.log; exit 1; }
cut -c1-500 $O/config4_tp1.json
timeout -k 10 420 python -u bench_suite.py e2e --n 10000 --runs 20 --clients 16 > $O/e2e.jsonl 2> $O/e2e.log || { echo "e2e failed"; tail -20 $O/e2e.log; exit 1; }
cut -c1-600 $O/e2e.jsonl
