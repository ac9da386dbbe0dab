set -o pipefail
mkdir -p gpurun_out/aab2
export TMPDIR=/tmp
for q in 40 80 120; do
for cfg in "1 -1" "0 -1" "1 4" "0 4"; do
set -- $cfg
MCP_CASCADE=$1 MCP_KV_SPLIT=$2 timeout -k 10 200 python -u bench_serve.py qps --qps $q --duration 12 > gpurun_out/aab2/q${q}_c$1_s$2.json 2> gpurun_out/aab2/q${q}_c$1_s$2.err || exit 1
echo "q=$q cascade=$1 split=$2 $(grep -o '"p50_latency_ms": [0-9.]*, "p99_latency_ms": [0-9.]*' gpurun_out/aab2/q${q}_c$1_s$2.json)"
done
done
