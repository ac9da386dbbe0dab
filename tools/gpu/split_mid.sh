set -o pipefail
mkdir -p gpurun_out/splitmid
export TMPDIR=/tmp
for S in 0 2 3 4 6 8; do
MCP_GEMM_SPLITK128=$S timeout -k 10 200 python -u tools/bench_small_m.py 256,320,384,448,512,640,768 > gpurun_out/splitmid/s$S.jsonl 2>&1 || exit 1
done
