set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 240 python -u tools/bench_small_m.py > gpurun_out/small_m.log 2>&1 && \
timeout -k 10 300 python -u tools/tune_gemm_plan.py gpurun_out/gemm_plan_gfx950.json 8192 > gpurun_out/tune.log 2>&1 && \
cp gpurun_out/gemm_plan_gfx950.json autonomous-microservice-composition-via-llm-agents-in-an-mcp-control-plane_amd/ops/gemm_plan_gfx950.json && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench2.log 2>&1
