#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4c}
mkdir -p $O
timeout -k 10 400 python -u tools/bench_gemm_group.py $O/group.jsonl > $O/group.log 2>&1 || { echo "group sweep failed"; tail -5 $O/group.log; exit 1; }
cat $O/group.jsonl | cut -c1-400
timeout -k 10 300 python -u tools/bench_gemm_mix.py tools/gemm_trace_bench_r4.jsonl 256 > $O/mix.jsonl 2> $O/mix.log || { echo "mix failed"; tail -5 $O/mix.log; exit 1; }
tail -4 $O/mix.jsonl
