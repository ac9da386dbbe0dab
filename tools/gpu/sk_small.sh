set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/bench_small_m.py 128,192,256,320,384,512 > gpurun_out/small_m_default.jsonl 2>&1 || exit 1
MCP_GEMM_STREAMK=1 timeout -k 10 200 python -u tools/bench_small_m.py 128,192,256,320,384,512 > gpurun_out/small_m_sk.jsonl 2>&1 || exit 1
