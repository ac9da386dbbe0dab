set -o pipefail
mkdir -p gpurun_out/rw
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "cascade_prefix" > gpurun_out/rw/tests.log 2>&1 || { tail -30 gpurun_out/rw/tests.log; exit 1; }
tail -2 gpurun_out/rw/tests.log
for S in 4 16 64 256; do
for ql in 4 12; do
for nw in 8 4 42 82; do
  MCP_PREFIX_SPLIT=0 MCP_ATTN_PREFIX_NW=$nw ATTN_S=$S ATTN_OWN=120 timeout -k 10 120 python -u tools/bench_attention.py $ql > gpurun_out/rw/one.json 2>gpurun_out/rw/err.txt || { tail -5 gpurun_out/rw/err.txt; exit 1; }
  echo "nw=$nw $(cat gpurun_out/rw/one.json)" | tee -a gpurun_out/rw/res.txt
done
done
done
