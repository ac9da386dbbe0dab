#!/bin/bash
# Flex tile x split-K: GPU numerics, tune the narrow shapes (qkv / o / down,
# every model and TP shard) at M <= 512, fold the "fsplit" buckets into a
# candidate plan, A/B config 5 (80 and 120 intents/s), alternated.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ax}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fsplit or flex or fused_norm" > $O/test.log 2>&1 || { echo "tests failed"; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
MCP_TUNE_SHAPES=narrow MCP_TUNE_COLD_ALL=1 timeout -k 10 900 python -u tools/tune_gemm_plan.py $O/plan_narrow.json 512 "8b+70b+8b-tp2+8b-tp4+8b-tp8+70b-tp2+70b-tp4+70b-tp8" > $O/tune.log 2>&1 || { echo "tune failed"; tail -5 $O/tune.log; exit 1; }
grep '^{"N"' $O/tune.log | cut -c1-330
CAND=tools/plan_fsplit_cand.json
cp autonomous-microservice-composition-via-llm-agents-in-an-mcp-control-plane_amd/ops/gemm_plan_gfx950.json $CAND
python tools/merge_gemm_plan.py $O/plan_narrow.json $CAND --keys fsplit > /dev/null && cp $CAND $O/ || exit 1
for v in ship cand ship cand; do
  if [ $v = cand ]; then export MCP_GEMM_PLAN=$CAND; else unset MCP_GEMM_PLAN; fi
  for q in 120 80; do
    timeout -k 10 300 python -u bench_serve.py qps --qps $q --duration 20 > $O/q${q}_$v.json 2> $O/q${q}_$v.log || { echo "qps $q $v failed"; tail -20 $O/q${q}_$v.log; exit 1; }
    echo "q$q $v $(cut -c1-330 $O/q${q}_$v.json)" | tee -a $O/ab.txt
  done
done
