#!/bin/bash
# Headline A/B of the grammar's compact model view (MCP_PLAN_COMPACT 1 / 0)
# on one box: bench.py at 10 timed steps, 3 warm-up, alternated.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4j}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/engine_tests.log 2>&1 || { echo "engine tests failed"; tail -30 $O/engine_tests.log; exit 1; }
tail -1 $O/engine_tests.log
for c in 1 0 1 0; do
  MCP_PLAN_COMPACT=$c timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench_c$c.json 2> $O/bench_c$c.log || { echo "bench c=$c failed"; tail -20 $O/bench_c$c.log; exit 1; }
  echo "compact=$c $(cut -c1-330 $O/bench_c$c.json)" | tee -a $O/ab.txt
done
