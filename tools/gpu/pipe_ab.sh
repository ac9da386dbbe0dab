set -o pipefail
mkdir -p gpurun_out/pipe
export TMPDIR=/tmp
for q in 40 80 160; do
  for p in 1 0; do
    MCP_PIPELINE=$p timeout -k 10 200 python -u bench_serve.py qps --qps $q --duration 10 > gpurun_out/pipe/q${q}_p${p}.json 2> gpurun_out/pipe/q${q}_p${p}.err || exit 1
    echo "q=$q pipe=$p $(cat gpurun_out/pipe/q${q}_p${p}.json)"
  done
done
