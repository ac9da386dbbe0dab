set -o pipefail
mkdir -p gpurun_out/rt
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/tune_gemm_plan.py gpurun_out/rt/plan.json > gpurun_out/rt/tune.log 2>&1 || { tail -20 gpurun_out/rt/tune.log; exit 1; }
tail -1 gpurun_out/rt/tune.log
for p in old new old new; do
  if [ $p = new ]; then export MCP_GEMM_PLAN=gpurun_out/rt/plan.json; else unset MCP_GEMM_PLAN; fi
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 > gpurun_out/rt/bench_$p.json 2> gpurun_out/rt/bench_$p.err || { tail -20 gpurun_out/rt/bench_$p.err; exit 1; }
  echo "$p $(cat gpurun_out/rt/bench_$p.json | cut -c1-200)"
done
