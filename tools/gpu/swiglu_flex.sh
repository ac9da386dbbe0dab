#!/bin/bash
# Flex SwiGLU epilogue: GPU numerics, then time the gate|up shapes (flex tiles
# with whole gate|up pairs per wave) for every model / TP shard, fold their
# "flex" buckets into a candidate plan and A/B it: config 5 at 120 intents/s
# and the headline, shipped vs candidate, alternated.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4as}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "flex" > $O/test.log 2>&1 || { echo "flex tests failed"; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
MCP_TUNE_SHAPES=swiglu MCP_TUNE_COLD_ALL=1 timeout -k 10 900 python -u tools/tune_gemm_plan.py $O/plan_swiglu.json 2048 "8b+70b+8b-tp2+8b-tp4+8b-tp8+70b-tp2+70b-tp4+70b-tp8" > $O/tune.log 2>&1 || { echo "tune failed"; tail -5 $O/tune.log; exit 1; }
cut -c1-400 $O/tune.log
CAND=tools/plan_swiglu_cand.json
cp autonomous-microservice-composition-via-llm-agents-in-an-mcp-control-plane_amd/ops/gemm_plan_gfx950.json $CAND
python tools/merge_gemm_plan.py $O/plan_swiglu.json $CAND --keys flex > /dev/null && cp $CAND $O/ || exit 1
for v in ship cand ship cand; do
  if [ $v = cand ]; then export MCP_GEMM_PLAN=$CAND; else unset MCP_GEMM_PLAN; fi
  timeout -k 10 300 python -u bench_serve.py qps --qps 120 --duration 20 > $O/q120_$v.json 2> $O/q120_$v.log || { echo "qps $v failed"; tail -20 $O/q120_$v.log; exit 1; }
  echo "q120 $v $(cut -c1-330 $O/q120_$v.json)" | tee -a $O/ab.txt
done
for v in ship cand ship cand; do
  if [ $v = cand ]; then export MCP_GEMM_PLAN=$CAND; else unset MCP_GEMM_PLAN; fi
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench_$v.json 2> $O/bench_$v.log || { echo "bench $v failed"; tail -20 $O/bench_$v.log; exit 1; }
  echo "head $v $(cut -c1-240 $O/bench_$v.json)" | tee -a $O/ab.txt
done
