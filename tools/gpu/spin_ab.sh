#!/bin/bash
# Config 2: busy-poll the sampled-token event vs hipEventSynchronize.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4an}
mkdir -p $O
for v in 0 1 0 1; do
  MCP_SPIN_WAIT=$v timeout -k 10 300 python -u bench_serve.py single --n 10 > $O/c2_$v.json 2> $O/c2_$v.log || { echo "config 2 $v failed"; tail -20 $O/c2_$v.log; exit 1; }
  echo "spin=$v $(cut -c1-400 $O/c2_$v.json)" | tee -a $O/ab.txt
done
