#!/bin/bash
# Headline A/B of the persistent AGPR GEMM on one box: bench.py (8 timed steps,
# 3 warm-up) alternating MCP_GEMM_PERSIST = 0 / 1 / 0 / 1.
# Usage (from the repo root, through gpurun): bash tools/gpu/persist_bench_ab.sh TAG
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4f}
mkdir -p $O
for p in 0 1 0 1; do
  MCP_GEMM_PERSIST=$p timeout -k 10 240 python -u bench.py --steps 8 --warmup 3 > $O/bench_p$p.json 2> $O/bench_p$p.log || { echo "bench p=$p failed"; tail -20 $O/bench_p$p.log; exit 1; }
  echo "persist=$p $(cut -c1-200 $O/bench_p$p.json)" | tee -a $O/ab.txt
done
