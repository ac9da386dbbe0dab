#!/bin/bash
# GEMM plan for the remaining TP shard shapes (70B at TP 2 / 4, 8B at TP 2 / 4 / 8).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4p}
mkdir -p $O
timeout -k 10 900 python -u tools/tune_gemm_plan.py $O/plan_tp_rest.json 4096 70b-tp2+70b-tp4+8b-tp2+8b-tp4+8b-tp8 > $O/tune.log 2>&1 || { echo "tune failed"; tail -5 $O/tune.log; exit 1; }
tail -2 $O/tune.log | cut -c1-300
