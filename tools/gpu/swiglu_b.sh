set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/bench_swiglu.py 2048,2432,2560,2624,2688,2752,2880,3072,4096 > gpurun_out/swiglu.jsonl 2>&1; cat gpurun_out/swiglu.jsonl
