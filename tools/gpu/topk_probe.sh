set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/topk_size_probe.py > gpurun_out/topk_size_probe.jsonl 2>&1; cat gpurun_out/topk_size_probe.jsonl
