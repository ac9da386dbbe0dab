#!/bin/bash
# rocprofv3 kernel trace of config 5 at 120 intents/s at HEAD.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ab}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f rocpd -d $O/prof -o run -- python -u bench_serve.py qps --qps 120 --duration 12 > $O/config5.json 2> $O/config5.log || { echo "rocprof failed"; tail -20 $O/config5.log; exit 1; }
cut -c1-300 $O/config5.json
