set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/mst.log
for t in 4096 8192 6144 4096 8192; do
  timeout -k 10 300 python -u bench.py --max-step-tokens $t > gpurun_out/mst_$t.log 2>&1 || exit 1
  grep '^{' gpurun_out/mst_$t.log | sed "s/^{/{\"mst\": $t, /" >> gpurun_out/mst.log
done
