set -o pipefail
cp autonomous-microservice-composition-via-llm-agents-in-an-mcp-control-plane_amd/ops/gemm_plan_gfx950.json gpurun_out/plan_lib.json
timeout -k 10 200 python -u tools/tune_gemm_lib.py gpurun_out/plan_lib.json > gpurun_out/tune_lib.log 2>&1
export MCP_GEMM_PLAN=gpurun_out/plan_lib.json
MCP_GEMM_LIB=1 timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 > gpurun_out/ab_lib1.log 2>&1
MCP_GEMM_LIB=0 timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 > gpurun_out/ab_lib0.log 2>&1
MCP_GEMM_LIB=1 timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 > gpurun_out/ab_lib1b.log 2>&1
tail -1 gpurun_out/ab_lib1.log gpurun_out/ab_lib0.log gpurun_out/ab_lib1b.log | cut -c1-200
