set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/small_m.log
for e in 0 1; do
  MCP_GEMM_SPLITK128=$e timeout -k 10 240 python -u tools/bench_small_m.py >> gpurun_out/small_m.log 2>&1 || exit 1
done
