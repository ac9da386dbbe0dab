set -o pipefail
mkdir -p gpurun_out/sweep2
for cfg in ${SWEEP:-"256 4096" "384 4096" "512 4096" "512 8192"}; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --batch $1 --max-step-tokens $2 > gpurun_out/sweep2/b$1_t$2.log 2>&1 || exit 1
done
