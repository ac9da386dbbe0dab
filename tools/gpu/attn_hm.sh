set -o pipefail
mkdir -p gpurun_out/hm
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "cascade_prefix" > gpurun_out/hm/tests.log 2>&1 || { tail -30 gpurun_out/hm/tests.log; exit 1; }
tail -2 gpurun_out/hm/tests.log
for S in 16 64 256; do
for ql in 4 12 16; do
for hm in 0 1; do
  MCP_PREFIX_SPLIT=0 MCP_ATTN_PREFIX_HEAD_MAJOR=$hm ATTN_S=$S ATTN_OWN=120 timeout -k 10 120 python -u tools/bench_attention.py $ql > gpurun_out/hm/one.json 2>gpurun_out/hm/err.txt || { tail -5 gpurun_out/hm/err.txt; exit 1; }
  echo "hm=$hm $(cut -c1-110 gpurun_out/hm/one.json)" | tee -a gpurun_out/hm/res.txt
done
done
done
