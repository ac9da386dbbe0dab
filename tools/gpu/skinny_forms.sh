#!/bin/bash
# Skinny kernel forms (waves x ring depth) after the load-order fix: numerics
# under each form, cold-weight timing, config 2.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4at}
mkdir -p $O
for f in 1 2 3; do
  MCP_GEMM_SKINNY_FORM=$f timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "skinny" > $O/test_$f.log 2>&1 || { echo "tests form $f failed"; tail -30 $O/test_$f.log; exit 1; }
  tail -1 $O/test_$f.log
done
for f in 0 1 2 3; do
  PROBE_TAG=form$f MCP_GEMM_SKINNY_FORM=$f timeout -k 10 400 python -u tools/bench_decode_probe.py >> $O/probe.jsonl 2>> $O/probe.log || { echo "probe $f failed"; tail -20 $O/probe.log; exit 1; }
done
python - <<'PY' $O/probe.jsonl
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(r["tag"], r["N"], r["K"], r["M"], r.get("skinny_us"), r["auto_us"])
PY
for f in 0 1 3 0 1 3; do
  MCP_GEMM_SKINNY_FORM=$f timeout -k 10 300 python -u bench_serve.py single --n 10 > $O/c2_$f.json 2> $O/c2_$f.log || { echo "config 2 $f failed"; tail -20 $O/c2_$f.log; exit 1; }
  echo "form=$f $(cut -c1-330 $O/c2_$f.json)" | tee -a $O/ab.txt
done
