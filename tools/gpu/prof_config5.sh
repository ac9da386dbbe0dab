#!/bin/bash
# rocprofv3 kernel trace of config 5 at 120 intents/s at HEAD; summarised on
# the box (the trace database exceeds what gpurun copies back).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ab}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f rocpd -d /tmp/prof5 -o run -- python -u bench_serve.py qps --qps 120 --duration 12 > $O/config5.json 2> $O/config5.log || { echo "rocprof failed"; tail -20 $O/config5.log; exit 1; }
cut -c1-300 $O/config5.json
python tools/rocpd_summary.py /tmp/prof5/run_results.db 6000 > $O/summary.md 2>&1 || { echo "summary failed"; tail -5 $O/summary.md; exit 1; }
head -40 $O/summary.md
