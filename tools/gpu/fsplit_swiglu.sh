#!/bin/bash
# Flex x split-K for gate|up (the reduce applies the SwiGLU): numerics, tune
# the TP=1 gate|up shapes up to M = 1024, A/B config 5 / config 4 / headline.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4az}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "swiglu or fsplit" > $O/test.log 2>&1 || { echo "tests failed"; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
MCP_TUNE_FS_MAX=1024 MCP_TUNE_SHAPES=swiglu MCP_TUNE_COLD_ALL=1 timeout -k 10 900 python -u tools/tune_gemm_plan.py $O/plan_swiglu.json 1024 "8b+70b" > $O/tune.log 2>&1 || { echo "tune failed"; tail -5 $O/tune.log; exit 1; }
grep '^{"N"' $O/tune.log | cut -c1-400
CAND=tools/plan_fsplit3_cand.json
cp autonomous-microservice-composition-via-llm-agents-in-an-mcp-control-plane_amd/ops/gemm_plan_gfx950.json $CAND
python tools/merge_gemm_plan.py $O/plan_swiglu.json $CAND --keys fsplit > /dev/null && cp $CAND $O/ || exit 1
for v in ship cand ship cand; do
  if [ $v = cand ]; then export MCP_GEMM_PLAN=$CAND; else unset MCP_GEMM_PLAN; fi
  timeout -k 10 300 python -u bench_serve.py qps --qps 120 --duration 20 > $O/q120_$v.json 2> $O/q120_$v.log || { echo "qps $v failed"; tail -20 $O/q120_$v.log; exit 1; }
  echo "q120 $v $(cut -c1-330 $O/q120_$v.json)" | tee -a $O/ab.txt
  timeout -k 10 500 python -u bench_tp.py --gpus 1 > $O/c4_$v.json 2> $O/c4_$v.log || { echo "config 4 $v failed"; tail -20 $O/c4_$v.log; exit 1; }
  echo "c4 $v $(cut -c1-300 $O/c4_$v.json)" | tee -a $O/ab.txt
done
