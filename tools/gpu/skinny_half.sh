#!/bin/bash
# SwiGLU skinny forms: GPU numerics, cold-weight timing, config 2 A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4af}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "skinny" > $O/test.log 2>&1 || { echo "skinny tests failed"; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python -u tools/bench_swiglu_decode.py > $O/swiglu.jsonl 2> $O/swiglu.log || { echo "bench failed"; tail -20 $O/swiglu.log; exit 1; }
cat $O/swiglu.jsonl
for v in 1 0 1 0; do
  MCP_GEMM_SKINNY_HALF=$v timeout -k 10 300 python -u bench_serve.py single --n 10 > $O/c2_$v.json 2> $O/c2_$v.log || { echo "config 2 $v failed"; tail -20 $O/c2_$v.log; exit 1; }
  echo "half=$v $(cut -c1-400 $O/c2_$v.json)" | tee -a $O/ab.txt
done
