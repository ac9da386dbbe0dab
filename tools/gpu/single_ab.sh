set -o pipefail
mkdir -p gpurun_out/sab
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_edge_cases_gpu.py -k "gemm or skinny or nan or silu" -x -q --timeout 200 --timeout-method thread > gpurun_out/sab/tests.log 2>&1 || { tail -30 gpurun_out/sab/tests.log; exit 1; }
tail -1 gpurun_out/sab/tests.log
for cfg in "1 -1 0" "1 -1 1" "0 -1 1" "0 4 1" "0 8 1"; do
set -- $cfg
MCP_CASCADE=$1 MCP_KV_SPLIT=$2 MCP_GEMM_SKINNY_FIRST=$3 timeout -k 10 300 python -u bench_serve.py single --n 12 > gpurun_out/sab/c$1_s$2_k$3.json 2> gpurun_out/sab/c$1_s$2_k$3.err || exit 1
echo "cascade=$1 split=$2 skinny=$3 $(grep -o '"p50_warm_prefix_ms": [0-9.]*, "p90_warm_prefix_ms": [0-9.]*, "p50_cold_prefix_ms": [0-9.]*' gpurun_out/sab/c$1_s$2_k$3.json)"
done
