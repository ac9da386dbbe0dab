#!/bin/bash
# Flex x split-K up to M = 1024 on the TP=1 narrow shapes (8B, 70B): tune,
# fold "fsplit" into a candidate, A/B config 4 (70B TP1), config 5 at 120/s
# and the headline, alternated.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ay}
mkdir -p $O
MCP_TUNE_FS_MAX=1024 MCP_TUNE_SHAPES=narrow MCP_TUNE_COLD_ALL=1 timeout -k 10 900 python -u tools/tune_gemm_plan.py $O/plan_narrow.json 1024 "8b+70b" > $O/tune.log 2>&1 || { echo "tune failed"; tail -5 $O/tune.log; exit 1; }
grep '^{"N"' $O/tune.log | cut -c1-400
CAND=tools/plan_fsplit2_cand.json
cp autonomous-microservice-composition-via-llm-agents-in-an-mcp-control-plane_amd/ops/gemm_plan_gfx950.json $CAND
python tools/merge_gemm_plan.py $O/plan_narrow.json $CAND --keys fsplit > /dev/null && cp $CAND $O/ || exit 1
for v in ship cand ship cand; do
  if [ $v = cand ]; then export MCP_GEMM_PLAN=$CAND; else unset MCP_GEMM_PLAN; fi
  timeout -k 10 500 python -u bench_tp.py --gpus 1 > $O/c4_$v.json 2> $O/c4_$v.log || { echo "config 4 $v failed"; tail -20 $O/c4_$v.log; exit 1; }
  echo "c4 $v $(cut -c1-300 $O/c4_$v.json)" | tee -a $O/ab.txt
  timeout -k 10 300 python -u bench_serve.py qps --qps 120 --duration 20 > $O/q120_$v.json 2> $O/q120_$v.log || { echo "qps $v failed"; tail -20 $O/q120_$v.log; exit 1; }
  echo "q120 $v $(cut -c1-330 $O/q120_$v.json)" | tee -a $O/ab.txt
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench_$v.json 2> $O/bench_$v.log || { echo "bench $v failed"; tail -20 $O/bench_$v.log; exit 1; }
  echo "head $v $(cut -c1-240 $O/bench_$v.json)" | tee -a $O/ab.txt
done
