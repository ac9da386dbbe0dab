#!/bin/bash
# New GPU tests of this round, config 3 end to end (block-level prefix reuse),
# config 5 direct vs through the HTTP front end.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4d}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "selfcheck or cascade_fold or large_rows" > $O/new_tests.log 2>&1 || { echo "new tests failed"; tail -30 $O/new_tests.log; exit 1; }
tail -1 $O/new_tests.log
timeout -k 10 420 python -u bench_suite.py e2e --n 10000 --runs 20 --clients 16 > $O/e2e.jsonl 2> $O/e2e.log || { echo "e2e failed"; tail -20 $O/e2e.log; exit 1; }
cut -c1-400 $O/e2e.jsonl
timeout -k 10 240 python -u bench_serve.py qps --qps 80 --duration 20 > $O/qps80_direct.json 2> $O/qps80_direct.log || { echo "qps direct failed"; tail -20 $O/qps80_direct.log; exit 1; }
cut -c1-300 $O/qps80_direct.json
MCP_SERVER_LOG=$O/server_r1.log timeout -k 10 420 python -u bench_serve.py qps --via-api --replicas 1 --qps 80 --duration 20 > $O/qps80_api_r1.json 2> $O/qps80_api_r1.log || { echo "qps api r1 failed"; tail -20 $O/qps80_api_r1.log; tail -20 $O/server_r1.log; exit 1; }
cat $O/qps80_api_r1.json
MCP_SERVER_LOG=$O/server_r0.log timeout -k 10 420 python -u bench_serve.py qps --via-api --replicas 0 --qps 80 --duration 20 > $O/qps80_api_r0.json 2> $O/qps80_api_r0.log || { echo "qps api r0 failed"; tail -20 $O/qps80_api_r0.log; tail -20 $O/server_r0.log; exit 1; }
cat $O/qps80_api_r0.json
