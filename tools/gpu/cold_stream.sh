set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/bench_cold_stream.py > gpurun_out/cold_stream.jsonl 2>&1; cat gpurun_out/cold_stream.jsonl
