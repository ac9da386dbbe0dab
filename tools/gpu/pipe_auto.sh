set -o pipefail
mkdir -p gpurun_out/pauto
export TMPDIR=/tmp
for q in 40 120 160 200; do
  timeout -k 10 300 python -u bench_serve.py qps --qps $q --duration 15 > gpurun_out/pauto/qps_$q.json 2> gpurun_out/pauto/qps_$q.err || exit 1
  echo "q=$q $(cat gpurun_out/pauto/qps_$q.json)"
done
