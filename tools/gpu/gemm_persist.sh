#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4e}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_persistent_gpu.py -x -q --timeout 120 --timeout-method thread > $O/persist_tests.log 2>&1 || { echo "persistent tests failed"; tail -40 $O/persist_tests.log; exit 1; }
tail -1 $O/persist_tests.log
timeout -k 10 400 python -u tools/bench_gemm_persist.py $O/persist.jsonl > $O/persist.log 2>&1 || { echo "persist bench failed"; tail -5 $O/persist.log; exit 1; }
cut -c1-300 $O/persist.jsonl
