set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_bench
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run -- python3 bench.py --steps 4 --warmup 2 > gpurun_out/prof_bench/bench.log 2>&1
python3 tools/rocpd_summary.py $(ls gpurun_out/prof_bench/*.db | head -1) 5100 > gpurun_out/prof_bench_summary.md
tail -3 gpurun_out/prof_bench/bench.log
rm -rf gpurun_out/prof_bench/*.db gpurun_out/prof_bench/*/
