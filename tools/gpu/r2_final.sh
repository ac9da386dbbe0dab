set -o pipefail
mkdir -p gpurun_out/r2f
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2f/gputests.log 2>&1 || { tail -40 gpurun_out/r2f/gputests.log; exit 1; }
tail -1 gpurun_out/r2f/gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2f/smoke.log 2>&1 || { tail -20 gpurun_out/r2f/smoke.log; exit 1; }
tail -1 gpurun_out/r2f/smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2f/bench.json 2> gpurun_out/r2f/bench.err && cat gpurun_out/r2f/bench.json
