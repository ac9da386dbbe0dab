#!/bin/bash
# Round-4 closing run: every GPU test, smoke(), the headline at the driver's
# shape, the BASELINE configs, and a timed-window rocprof of the headline
# summarised on the box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4av}
mkdir -p $O
bash tools/gpu/final_check.sh $1 || exit 1
bash tools/gpu/final_configs.sh $1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f rocpd -d $O/prof -o run -- python -u bench.py --steps 4 --warmup 1 > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
python tools/rocpd_summary.py $O/prof/run_results.db 3300 > $O/rocprof_head.md && rm -f $O/prof/run_results.db
head -30 $O/rocprof_head.md
