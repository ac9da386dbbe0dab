#!/bin/bash
# Headline A/B of the engine's step token budget (bench.py --max-step-tokens).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4aa}
mkdir -p $O
for t in 4096 8192 4096 8192 3072; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --max-step-tokens $t > $O/bench_t$t.json 2> $O/bench_t$t.log || { echo "bench t=$t failed"; tail -20 $O/bench_t$t.log; exit 1; }
  echo "tokens=$t $(cut -c1-200 $O/bench_t$t.json)" | tee -a $O/ab.txt
done
