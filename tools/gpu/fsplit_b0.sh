#!/bin/bash
# Flex x split-K for bucket 0 (M 33-64 reach it once the stream / skinny
# kernels decline): tune at M = 64 for the TP=1 shapes, A/B config 5 at 80 / 40
# intents/s and config 2, alternated.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4bi}
mkdir -p $O
MCP_TUNE_FS_MIN=1 MCP_TUNE_COLD_ALL=1 timeout -k 10 600 python -u tools/tune_gemm_plan.py $O/plan_b0.json 64 "8b+70b" > $O/tune.log 2>&1 || { echo "tune failed"; tail -5 $O/tune.log; exit 1; }
grep '^{"N"' $O/tune.log | cut -c1-300
CAND=tools/plan_fsplit_b0_cand.json
cp autonomous-microservice-composition-via-llm-agents-in-an-mcp-control-plane_amd/ops/gemm_plan_gfx950.json $CAND
python tools/merge_gemm_plan.py $O/plan_b0.json $CAND --keys fsplit > /dev/null && cp $CAND $O/ || exit 1
for v in ship cand ship cand; do
  if [ $v = cand ]; then export MCP_GEMM_PLAN=$CAND; else unset MCP_GEMM_PLAN; fi
  for q in 80 40; do
    timeout -k 10 300 python -u bench_serve.py qps --qps $q --duration 20 > $O/q${q}_$v.json 2> $O/q${q}_$v.log || { echo "qps $q $v failed"; tail -20 $O/q${q}_$v.log; exit 1; }
    echo "q$q $v $(cut -c1-330 $O/q${q}_$v.json)" | tee -a $O/ab.txt
  done
  timeout -k 10 300 python -u bench_serve.py single --n 10 > $O/c2_$v.json 2> $O/c2_$v.log || { echo "config 2 $v failed"; tail -20 $O/c2_$v.log; exit 1; }
  echo "c2 $v $(cut -c1-330 $O/c2_$v.json)" | tee -a $O/ab.txt
done
