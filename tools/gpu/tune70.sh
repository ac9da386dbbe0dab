set -o pipefail
P=autonomous-microservice-composition-via-llm-agents-in-an-mcp-control-plane_amd/ops/gemm_plan_gfx950.json
cp $P gpurun_out/plan_merged.json
timeout -k 10 600 python -u tools/tune_gemm_plan.py gpurun_out/plan70.json 4096 70b > gpurun_out/tune70.log 2>&1 || { tail -5 gpurun_out/tune70.log; exit 1; }
python tools/merge_gemm_plan.py gpurun_out/plan70.json gpurun_out/plan_merged.json
MCP_GEMM_PLAN=gpurun_out/plan_merged.json timeout -k 10 300 python -u tools/tune_gemm_lib.py gpurun_out/plan_merged.json 4096 8192x8192,8192x28672,10240x8192 > gpurun_out/tune70_lib.log 2>&1 || { tail -5 gpurun_out/tune70_lib.log; exit 1; }
tail -n 2 gpurun_out/tune70_lib.log | cut -c1-200
for plan in gpurun_out/plan_merged.json $P; do
  MCP_GEMM_PLAN=$plan timeout -k 10 600 python -u bench_tp.py --steps 3 --warmup 1 > gpurun_out/c4_$(basename $plan .json).json 2> gpurun_out/c4_$(basename $plan .json).err || { tail -5 gpurun_out/c4_$(basename $plan .json).err; exit 1; }
  echo "$plan $(cat gpurun_out/c4_$(basename $plan .json).json | cut -c1-300)"
done
