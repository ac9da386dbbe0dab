#!/bin/bash
# rocprofv3 kernel trace of config 2 (single intent, graphs) at HEAD.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4u}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f rocpd -d $O/prof -o run -- python -u bench_serve.py single --n 10 > $O/config2.json 2> $O/config2.log || { echo "rocprof failed"; tail -20 $O/config2.log; exit 1; }
cut -c1-300 $O/config2.json
