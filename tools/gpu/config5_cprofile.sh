#!/bin/bash
# Host-side profile of config 5 at 120 intents/s.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ar}
mkdir -p $O
timeout -k 10 300 python -u -m cProfile -o $O/q120.prof bench_serve.py qps --qps 120 --duration 15 > $O/q120.json 2> $O/q120.log || { echo "qps failed"; tail -20 $O/q120.log; exit 1; }
cut -c1-300 $O/q120.json
