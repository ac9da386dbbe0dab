#!/bin/bash
# Config 5 at 160 / 200 intents/s (one GPU) at HEAD.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4y}
mkdir -p $O
for q in 160 200 240; do
  timeout -k 10 300 python -u bench_serve.py qps --qps $q --duration 20 > $O/config5_q$q.json 2> $O/config5_q$q.log || { echo "config 5 q$q failed"; tail -20 $O/config5_q$q.log; exit 1; }
  cut -c1-330 $O/config5_q$q.json
done
