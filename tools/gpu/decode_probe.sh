#!/bin/bash
# Decode-sized projections at single-intent M, cold weights: shipped dispatch,
# forced stream splits; then the skinny X-row probe.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ag}
mkdir -p $O
PROBE_TAG=ship timeout -k 10 400 python -u tools/bench_decode_probe.py > $O/probe.jsonl 2> $O/probe.log || { echo "probe failed"; tail -20 $O/probe.log; exit 1; }
PROBE_TAG=x1 MCP_PROBE_SKINNY_X1=1 timeout -k 10 400 python -u tools/bench_decode_probe.py >> $O/probe.jsonl 2>> $O/probe.log || { echo "probe x1 failed"; tail -20 $O/probe.log; exit 1; }
cat $O/probe.jsonl
