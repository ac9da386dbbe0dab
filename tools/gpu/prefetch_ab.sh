#!/bin/bash
# Infinity Cache weight prefetch beside the decode attention: numerics, then
# config 2 A/B (off / 64 MB / 40 MB per layer), alternated.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ao}
mkdir -p $O
MCP_WEIGHT_PREFETCH=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "prefetch or engine" > $O/test.log 2>&1 || { echo "tests failed"; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for v in 0 64 40 0 64 40; do
  if [ $v = 0 ]; then P=0; else P=1; fi
  MCP_WEIGHT_PREFETCH=$P MCP_WEIGHT_PREFETCH_MB=$v timeout -k 10 300 python -u bench_serve.py single --n 10 > $O/c2_$v.json 2> $O/c2_$v.log || { echo "config 2 $v failed"; tail -20 $O/c2_$v.log; exit 1; }
  echo "prefetch_mb=$v $(cut -c1-400 $O/c2_$v.json)" | tee -a $O/ab.txt
done
