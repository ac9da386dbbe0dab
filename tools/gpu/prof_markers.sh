set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/profm
export MCP_ROCTX=1
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace -d gpurun_out/profm -o run -- python3 bench.py --steps 2 > gpurun_out/profm/bench.log 2>&1
