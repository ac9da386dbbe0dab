#!/bin/bash
# GEMM (M, N, K) histogram of config 5 at 120 intents/s (eager calls; graph
# captures counted once at capture).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4aq}
mkdir -p $O
MCP_GEMM_TRACE=$O/mhist.jsonl timeout -k 10 300 python -u bench_serve.py qps --qps 120 --duration 20 > $O/q120.json 2> $O/q120.log || { echo "qps failed"; tail -20 $O/q120.log; exit 1; }
cut -c1-300 $O/q120.json
wc -l $O/mhist.jsonl
timeout -k 10 400 python -u tools/bench_midm_probe.py > $O/midm.jsonl 2> $O/midm.log || { echo "midm probe failed"; tail -20 $O/midm.log; exit 1; }
cut -c1-260 $O/midm.jsonl
