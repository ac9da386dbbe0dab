set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pq40
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pq40 -o run -- python3 bench_serve.py qps --qps 40 --duration 8 > gpurun_out/pq40/serve.log 2>&1
python3 tools/rocpd_summary.py gpurun_out/pq40/run_results.db 6000 > gpurun_out/pq40_summary.md
rm -rf gpurun_out/pq40/*.db gpurun_out/pq40/*/
