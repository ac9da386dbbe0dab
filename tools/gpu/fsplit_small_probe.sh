#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4be}
mkdir -p $O
PROBE_MS=8,16,32,64 PROBE_WIDE=1 timeout -k 10 600 python -u tools/bench_flex_split_probe.py > $O/probe.jsonl 2> $O/probe.log || { echo "probe failed"; tail -20 $O/probe.log; exit 1; }
cat $O/probe.jsonl
