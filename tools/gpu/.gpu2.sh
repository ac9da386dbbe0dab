set -o pipefail
mkdir -p gpurun_out/sweep
for cfg in "256 8192" "384 8192" "512 8192" "512 4096"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --batch $1 --max-step-tokens $2 > gpurun_out/sweep/b$1_t$2.log 2>&1 || exit 1
done
