#!/bin/bash
# Flex x split-K at large M (up to 4096) on the 8B narrow shapes; headline A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4bb}
mkdir -p $O
MCP_TUNE_FS_MAX=4096 MCP_TUNE_SHAPES=narrow MCP_TUNE_COLD_ALL=1 timeout -k 10 1000 python -u tools/tune_gemm_plan.py $O/plan_big.json 4096 "8b" > $O/tune.log 2>&1 || { echo "tune failed"; tail -5 $O/tune.log; exit 1; }
grep '^{"N"' $O/tune.log | cut -c1-700
CAND=tools/plan_fsplit5_cand.json
cp autonomous-microservice-composition-via-llm-agents-in-an-mcp-control-plane_amd/ops/gemm_plan_gfx950.json $CAND
python tools/merge_gemm_plan.py $O/plan_big.json $CAND --keys fsplit > /dev/null && cp $CAND $O/ || exit 1
for v in ship cand ship cand; do
  if [ $v = cand ]; then export MCP_GEMM_PLAN=$CAND; else unset MCP_GEMM_PLAN; fi
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench_$v.json 2> $O/bench_$v.log || { echo "bench $v failed"; tail -20 $O/bench_$v.log; exit 1; }
  echo "head $v $(cut -c1-240 $O/bench_$v.json)" | tee -a $O/ab.txt
done
