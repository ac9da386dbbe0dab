set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_bench gpurun_out/prof_q80
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run -- python3 bench.py --steps 4 --warmup 2 > gpurun_out/prof_bench/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q80 -o run -- python3 bench_serve.py qps --qps 80 --duration 10 > gpurun_out/prof_q80/serve.log 2>&1
ls -la gpurun_out/prof_bench gpurun_out/prof_q80 > gpurun_out/prof_ls.txt
python3 tools/rocpd_summary.py $(ls gpurun_out/prof_bench/*.db | head -1) > gpurun_out/prof_bench_summary.md
python3 tools/rocpd_summary.py $(ls gpurun_out/prof_q80/*.db | head -1) > gpurun_out/prof_q80_summary.md
tail -3 gpurun_out/prof_bench/bench.log gpurun_out/prof_q80/serve.log
rm -rf gpurun_out/prof_bench/*.db gpurun_out/prof_q80/*.db gpurun_out/prof_bench/*/ gpurun_out/prof_q80/*/
