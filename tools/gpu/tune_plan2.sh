set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/tune_gemm_plan.py gpurun_out/gemm_plan_gfx950.json > gpurun_out/tune_plan.log 2>&1 || { tail -20 gpurun_out/tune_plan.log; exit 1; }
tail -6 gpurun_out/tune_plan.log
