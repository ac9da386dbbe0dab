#!/bin/bash
# Host-side profile of config 2 (single intent): where the per-step CPU time goes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4am}
mkdir -p $O
timeout -k 10 300 python -u -m cProfile -o $O/c2.prof bench_serve.py single --n 10 > $O/c2.json 2> $O/c2.log || { echo "config 2 failed"; tail -20 $O/c2.log; exit 1; }
cut -c1-300 $O/c2.json
