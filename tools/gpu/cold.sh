set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_cold_small_m.py > gpurun_out/cold_small_m.jsonl 2>&1; cat gpurun_out/cold_small_m.jsonl
