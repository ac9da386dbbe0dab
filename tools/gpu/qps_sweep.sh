set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/qps_sweep.log
for q in ${QPS_LIST:-20 40 80 120 160}; do
  timeout -k 10 300 python -u bench_serve.py qps --qps $q --duration 15 > gpurun_out/qps_$q.log 2>&1 || exit 1
  grep '^{' gpurun_out/qps_$q.log >> gpurun_out/qps_sweep.log
done
