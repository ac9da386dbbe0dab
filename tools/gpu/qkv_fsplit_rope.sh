#!/bin/bash
# QKV through flex x split-K with RoPE / K-V write fused into the reduce:
# numerics, then config 5 at 120 intents/s and 80 (MCP_QKV_ROPE_FSPLIT 1 vs 0).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4bf}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "qkv or rope or fsplit or engine" > $O/test.log 2>&1 || { echo "tests failed"; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for v in 1 0 1 0; do
  for q in 120 80; do
    MCP_QKV_ROPE_FSPLIT=$v timeout -k 10 300 python -u bench_serve.py qps --qps $q --duration 20 > $O/q${q}_$v.json 2> $O/q${q}_$v.log || { echo "qps $q $v failed"; tail -20 $O/q${q}_$v.log; exit 1; }
    echo "q$q rope_fsplit=$v $(cut -c1-330 $O/q${q}_$v.json)" | tee -a $O/ab.txt
  done
done
