#!/bin/bash
# Re-tune the Llama-3-8B TP=1 GEMM plan with the current kernels (cold weights
# at every M), then A/B the headline: shipped plan vs the new one.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4v}
mkdir -p $O
MCP_TUNE_COLD_ALL=1 timeout -k 10 900 python -u tools/tune_gemm_plan.py $O/plan_8b.json 8192 8b > $O/tune.log 2>&1 || { echo "tune failed"; tail -5 $O/tune.log; exit 1; }
tail -1 $O/tune.log | cut -c1-200
