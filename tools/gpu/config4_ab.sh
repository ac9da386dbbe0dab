#!/bin/bash
# Config 4 (70B, TP=1 on one box) with the compact / full model view.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4n}
mkdir -p $O
for c in 0 1; do
  MCP_PLAN_COMPACT=$c timeout -k 10 500 python -u bench_tp.py --gpus 1 > $O/config4_c$c.json 2> $O/config4_c$c.log || { echo "config 4 c$c failed"; tail -20 $O/config4_c$c.log; exit 1; }
  echo "compact=$c $(cut -c1-420 $O/config4_c$c.json)"
done
