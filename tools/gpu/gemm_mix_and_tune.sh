#!/bin/bash
# GEMM efficiency at the headline's own shapes (replay of the bench's GEMM
# trace, cold weights, ours vs hipBLASLt) and the GEMM plan for TP shard shapes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4b}
mkdir -p $O
timeout -k 10 300 python -u tools/bench_gemm_mix.py tools/gemm_trace_bench_r4.jsonl 256 > $O/mix.jsonl 2> $O/mix.log || { echo "mix failed"; tail -5 $O/mix.log; exit 1; }
tail -4 $O/mix.jsonl
timeout -k 10 600 python -u tools/tune_gemm_plan.py $O/plan_70b_tp8.json 4096 70b-tp8 > $O/tune_70b_tp8.log 2>&1 || { echo "tune failed"; tail -5 $O/tune_70b_tp8.log; exit 1; }
tail -3 $O/tune_70b_tp8.log
