#!/bin/bash
# Config 5 at 120 intents/s: hipGraph steps up to 128 (default) / 256 / 512 tokens.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ac}
mkdir -p $O
for t in 128 256 512 128; do
  MCP_GRAPH_MAX_TOKENS=$t timeout -k 10 300 python -u bench_serve.py qps --qps 120 --duration 20 > $O/q120_g$t.json 2> $O/q120_g$t.log || { echo "qps g$t failed"; tail -20 $O/q120_g$t.log; exit 1; }
  echo "graph_max=$t $(cut -c1-330 $O/q120_g$t.json)" | tee -a $O/ab.txt
done
