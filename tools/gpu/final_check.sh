#!/bin/bash
# Round-end rehearsal: every GPU test, smoke(), the headline at the driver's shape.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4x}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.log || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
cut -c1-400 $O/bench.json
