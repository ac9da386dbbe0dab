set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/split_sweep.log
for e in 1 2 4 7 8; do
  MCP_GEMM_SPLITK_MB=256 MCP_GEMM_SPLITK128=$e timeout -k 10 200 python -u tools/bench_small_m.py 768,1024,1152,1536,2048 >> gpurun_out/split_sweep.log 2>&1 || exit 1
done
