#!/bin/bash
# HEAD check on one MI355X: GPU tests, the headline bench at the driver's shape,
# the bench's GEMM shape histogram, and a rocprofv3 kernel trace of a short bench.
# Usage (from the repo root, through gpurun): bash tools/gpu/head_check.sh TAG
set -o pipefail
TAG=${1:-head}
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.log || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
cat $O/bench.json
MCP_GEMM_TRACE=$O/gemm_trace.jsonl timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 > $O/bench_trace.json 2> $O/bench_trace.log || { echo "trace run failed"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f rocpd -d $O/prof -o run -- python -u bench.py --steps 4 --warmup 1 > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
echo done
