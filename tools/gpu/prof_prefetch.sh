#!/bin/bash
# Kernel trace of config 2 with the weight prefetch on (why it loses).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ap}
mkdir -p $O
MCP_WEIGHT_PREFETCH=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -f rocpd -d $O/prof -o run -- python -u bench_serve.py single --n 4 > $O/c2.json 2> $O/c2.log || { echo "rocprof failed"; tail -20 $O/c2.log; exit 1; }
cut -c1-300 $O/c2.json
