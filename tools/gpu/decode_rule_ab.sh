#!/bin/bash
# Stream split rule (about one workgroup per CU) + tall-K skinny-first
# exception vs the round-3 rule; SwiGLU skinny forms after the load-order fix.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ai}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { echo "tests failed"; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python -u tools/bench_swiglu_decode.py > $O/swiglu.jsonl 2> $O/swiglu.log || { echo "swiglu bench failed"; tail -20 $O/swiglu.log; exit 1; }
cat $O/swiglu.jsonl
for v in 1 0 1 0; do
  MCP_STREAM_SPLIT_RULE=$v timeout -k 10 300 python -u bench_serve.py single --n 10 > $O/c2_$v.json 2> $O/c2_$v.log || { echo "config 2 $v failed"; tail -20 $O/c2_$v.log; exit 1; }
  echo "rule=$v $(cut -c1-400 $O/c2_$v.json)" | tee -a $O/ab.txt
done
for v in 1 0; do
  MCP_GEMM_SKINNY_HALF=$v timeout -k 10 300 python -u bench_serve.py single --n 10 > $O/c2h_$v.json 2> $O/c2h_$v.log || { echo "config 2 half $v failed"; tail -20 $O/c2h_$v.log; exit 1; }
  echo "half=$v $(cut -c1-400 $O/c2h_$v.json)" | tee -a $O/ab.txt
done
