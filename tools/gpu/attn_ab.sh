set -o pipefail
mkdir -p gpurun_out/aab
export TMPDIR=/tmp
for cfg in "1 -1" "0 -1" "1 4" "0 4" "0 8"; do
set -- $cfg
MCP_CASCADE=$1 MCP_KV_SPLIT=$2 timeout -k 10 200 python -u bench_serve.py qps --qps 40 --duration 8 --no-graphs > gpurun_out/aab/c$1_s$2.json 2> gpurun_out/aab/c$1_s$2.err || exit 1
echo "cascade=$1 split=$2 $(cat gpurun_out/aab/c$1_s$2.json)"
done
