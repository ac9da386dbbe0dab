set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_splitkv_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "split or attention or engine or graph" > gpurun_out/attn2_tests.log 2>&1 || { tail -40 gpurun_out/attn2_tests.log; exit 1; }
tail -3 gpurun_out/attn2_tests.log
timeout -k 10 300 python -u tools/bench_attention_splitkv.py > gpurun_out/attn_splitkv_final.jsonl 2>&1; cat gpurun_out/attn_splitkv_final.jsonl
timeout -k 10 300 python -u bench_serve.py single --n 10 > gpurun_out/config2.json 2> gpurun_out/config2.err; cat gpurun_out/config2.json
