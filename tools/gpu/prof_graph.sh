set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pg gpurun_out/pe
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pg -o run -- python3 bench_serve.py qps --qps 40 --duration 6 > gpurun_out/pg/serve.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pe -o run -- python3 bench_serve.py qps --qps 40 --duration 6 --no-graphs > gpurun_out/pe/serve.log 2>&1
python3 tools/rocpd_summary.py gpurun_out/pg/run_results.db 6000 > gpurun_out/pg_summary.md
python3 tools/rocpd_summary.py gpurun_out/pe/run_results.db 6000 > gpurun_out/pe_summary.md
rm -rf gpurun_out/pg/*.db gpurun_out/pe/*.db gpurun_out/pg/*/ gpurun_out/pe/*/
