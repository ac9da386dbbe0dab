#!/bin/bash
# Decode attention: tiles per wave forced to 2 / 4 (fewer blocks to merge) vs
# the grid rule, config 2; numerics under the forced form first.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4al}
mkdir -p $O
MCP_ATTN_DECODE_TPW=2 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_splitkv_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "decode or split" > $O/test.log 2>&1 || { echo "tests failed"; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for v in 0 2 4 0 2 4; do
  MCP_ATTN_DECODE_TPW=$v timeout -k 10 300 python -u bench_serve.py single --n 10 > $O/c2_$v.json 2> $O/c2_$v.log || { echo "config 2 $v failed"; tail -20 $O/c2_$v.log; exit 1; }
  echo "tpw=$v $(cut -c1-400 $O/c2_$v.json)" | tee -a $O/ab.txt
done
