#!/bin/bash
# Skinny kernel with contiguous-per-instruction loads: numerics, cold timing
# (shipped dispatch; skinny for wide M <= 16), config 2 A/B vs the stream
# kernel for wide M 9..16.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ah}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "skinny or gemm_small or stream" > $O/test.log 2>&1 || { echo "tests failed"; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
PROBE_TAG=contig timeout -k 10 400 python -u tools/bench_decode_probe.py > $O/probe.jsonl 2> $O/probe.log || { echo "probe failed"; tail -20 $O/probe.log; exit 1; }
PROBE_TAG=contig_wide16 MCP_GEMM_SKINNY_WIDE_MAXM=16 timeout -k 10 400 python -u tools/bench_decode_probe.py >> $O/probe.jsonl 2>> $O/probe.log || { echo "probe w16 failed"; tail -20 $O/probe.log; exit 1; }
cut -c1-200 $O/probe.jsonl
for v in 8 16 8 16; do
  MCP_GEMM_SKINNY_WIDE_MAXM=$v timeout -k 10 300 python -u bench_serve.py single --n 10 > $O/c2_$v.json 2> $O/c2_$v.log || { echo "config 2 $v failed"; tail -20 $O/c2_$v.log; exit 1; }
  echo "wide_maxm=$v $(cut -c1-400 $O/c2_$v.json)" | tee -a $O/ab.txt
done
