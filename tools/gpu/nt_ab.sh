set -o pipefail
mkdir -p gpurun_out/nt
export TMPDIR=/tmp
for nt in 0 1 0 1; do
  MCP_GEMM_NT=$nt timeout -k 10 200 python -u tools/bench_gemm.py 2048,2816,4096 > gpurun_out/nt/g_$nt.jsonl 2>gpurun_out/nt/err.txt || { tail -5 gpurun_out/nt/err.txt; exit 1; }
  echo "nt=$nt"; cut -c1-140 gpurun_out/nt/g_$nt.jsonl
done
