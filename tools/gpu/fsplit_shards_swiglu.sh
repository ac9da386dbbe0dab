#!/bin/bash
# Flex x split-K up to M = 1024 on the TP shard gate|up shapes; A/B the
# simulated TP=8 rank of config 4 (70B), alternated.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4bd}
mkdir -p $O
MCP_TUNE_FS_MAX=1024 MCP_TUNE_SHAPES=swiglu MCP_TUNE_COLD_ALL=1 timeout -k 10 900 python -u tools/tune_gemm_plan.py $O/plan_shards_swiglu.json 1024 "70b-tp8+70b-tp4+70b-tp2+8b-tp2+8b-tp4+8b-tp8" > $O/tune.log 2>&1 || { echo "tune failed"; tail -5 $O/tune.log; exit 1; }
grep '^{"N"' $O/tune.log | cut -c1-400
CAND=tools/plan_fsplit6_cand.json
cp autonomous-microservice-composition-via-llm-agents-in-an-mcp-control-plane_amd/ops/gemm_plan_gfx950.json $CAND
python tools/merge_gemm_plan.py $O/plan_shards_swiglu.json $CAND --keys fsplit > /dev/null && cp $CAND $O/ || exit 1
for v in ship cand ship cand; do
  if [ $v = cand ]; then export MCP_GEMM_PLAN=$CAND; else unset MCP_GEMM_PLAN; fi
  timeout -k 10 600 python -u bench_tp.py --simulate-rank 8 --model llama3-70b --steps 2 --warmup 1 > $O/tp8_$v.json 2> $O/tp8_$v.log || { echo "simulate-rank $v failed"; tail -30 $O/tp8_$v.log; exit 1; }
  echo "tp8sim $v $(cut -c1-420 $O/tp8_$v.json)" | tee -a $O/ab.txt
done
