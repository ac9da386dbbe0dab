set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MCP_GEMM_TRACE=gpurun_out/gemm_trace_qps80.jsonl timeout -k 10 300 python -u bench_serve.py qps --qps 80 --duration 10 --no-graphs > gpurun_out/serve_qps80_nograph.json 2> gpurun_out/serve_qps80_nograph.err && \
timeout -k 10 300 python -u bench_serve.py qps --qps 80 --duration 10 > gpurun_out/serve_qps80.json 2> gpurun_out/serve_qps80.err && \
timeout -k 10 300 python -u tools/bench_small_m.py 16,32,48,64,96,128,192,256 > gpurun_out/small_m_base.jsonl 2>&1
