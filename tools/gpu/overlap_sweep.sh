set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/overlap.log
for o in 0.4 0 0.25 0.6 0.4 0; do
  timeout -k 10 300 python -u bench.py --overlap $o > gpurun_out/ov_$o.log 2>&1 || exit 1
  grep '^{' gpurun_out/ov_$o.log | sed "s/^{/{\"overlap\": $o, /" >> gpurun_out/overlap.log
done
