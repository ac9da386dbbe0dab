set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_final.log 2>&1 || { tail -30 gpurun_out/gputest_final.log; exit 1; }
tail -n 1 gpurun_out/gputest_final.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_final.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench_final.log | cut -c1-200
bash tools/gpu/prof_r2b.sh
QPS_LIST="20 40 80 120 160" bash tools/gpu/qps_sweep.sh || exit 1
cat gpurun_out/qps_sweep.log | cut -c1-260
timeout -k 10 300 python -u bench_serve.py single --n 16 > gpurun_out/single_final.json 2> gpurun_out/single_final.err || exit 1
cat gpurun_out/single_final.json
