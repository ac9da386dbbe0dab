set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/profb
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/profb -o run -- python3 bench.py ${BENCH_ARGS:-} > gpurun_out/profb/bench.log 2>&1
