set -o pipefail
mkdir -p gpurun_out/sks
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" > gpurun_out/sks/tests.log 2>&1 || { tail -30 gpurun_out/sks/tests.log; exit 1; }
tail -2 gpurun_out/sks/tests.log
for sk in 0 1; do
  MCP_GEMM_BM=256 MCP_GEMM_SK_SMALL=$sk timeout -k 10 200 python -u tools/bench_gemm.py 512,1024,1536,2048 > gpurun_out/sks/g_$sk.jsonl 2>gpurun_out/sks/err.txt || { tail -5 gpurun_out/sks/err.txt; exit 1; }
  echo "sk=$sk"; cut -c1-140 gpurun_out/sks/g_$sk.jsonl
done
