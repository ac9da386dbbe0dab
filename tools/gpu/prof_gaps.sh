set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/profm
export MCP_ROCTX=1
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace -d gpurun_out/profm -o run -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/profm/bench.log 2>&1
python3 tools/gap_attribution.py $(ls gpurun_out/profm/*.db | head -1) 3600 200 > gpurun_out/gap_attr.md
python3 tools/rocpd_summary.py $(ls gpurun_out/profm/*.db | head -1) 3600 > gpurun_out/profm_summary.md
tail -n 1 gpurun_out/profm/bench.log | cut -c1-200
rm -rf gpurun_out/profm/*.db gpurun_out/profm/*/
