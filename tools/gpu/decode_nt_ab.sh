#!/bin/bash
# Config 2 (single intent): non-temporal weight loads in the decode GEMMs
# (stream kernel MCP_GEMM_STREAM_NT, skinny kernel MCP_GEMM_SKINNY_NT), cold
# weights as a real decode step sees them; alternated.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ae}
mkdir -p $O
for v in 00 11 10 01 00 11; do
  MCP_GEMM_STREAM_NT=${v:0:1} MCP_GEMM_SKINNY_NT=${v:1:1} timeout -k 10 300 python -u bench_serve.py single --n 10 > $O/c2_$v.json 2> $O/c2_$v.log || { echo "config 2 $v failed"; tail -20 $O/c2_$v.log; exit 1; }
  echo "stream_nt=${v:0:1} skinny_nt=${v:1:1} $(cut -c1-400 $O/c2_$v.json)" | tee -a $O/ab.txt
done
