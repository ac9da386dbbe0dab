#!/bin/bash
# BASELINE configs 2, 5 and 4 (TP=1) at HEAD on one box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4l}
mkdir -p $O
timeout -k 10 300 python -u bench_serve.py single --n 20 > $O/config2.json 2> $O/config2.log || { echo "config 2 failed"; tail -20 $O/config2.log; exit 1; }
cut -c1-400 $O/config2.json
for q in 80 120; do
  timeout -k 10 300 python -u bench_serve.py qps --qps $q --duration 20 > $O/config5_q$q.json 2> $O/config5_q$q.log || { echo "config 5 q$q failed"; tail -20 $O/config5_q$q.log; exit 1; }
  cut -c1-400 $O/config5_q$q.json
done
timeout -k 10 600 python -u bench_tp.py --gpus 1 > $O/config4_tp1.json 2> $O/config4_tp1.log || { echo "config 4 failed"; tail -20 $O/config4_tp1.log; exit 1; }
cut -c1-500 $O/config4_tp1.json
