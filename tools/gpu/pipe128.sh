set -o pipefail
mkdir -p gpurun_out/p128
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm" -x -q --timeout 200 --timeout-method thread > gpurun_out/p128/tests0.log 2>&1 || { tail -30 gpurun_out/p128/tests0.log; exit 1; }
MCP_GEMM128_PIPE=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm" -x -q --timeout 200 --timeout-method thread > gpurun_out/p128/tests1.log 2>&1 || { tail -30 gpurun_out/p128/tests1.log; exit 1; }
tail -1 gpurun_out/p128/tests0.log gpurun_out/p128/tests1.log
for P in 0 1; do  # MCP_GEMM128_PIPE
for S in 0 2 4 8; do
MCP_GEMM128_PIPE=$P MCP_GEMM_SPLITK128=$S timeout -k 10 200 python -u tools/bench_small_m.py 128,192,256,384,512,640,768,1024 > gpurun_out/p128/p${P}_s$S.jsonl 2>&1 || exit 1
done
done
