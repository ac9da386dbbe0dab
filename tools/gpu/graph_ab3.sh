set -o pipefail
mkdir -p gpurun_out/gab
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gab/tests.log 2>&1 || { tail -40 gpurun_out/gab/tests.log; exit 1; }
tail -2 gpurun_out/gab/tests.log
for q in 40 80; do
timeout -k 10 200 python -u bench_serve.py qps --qps $q --duration 10 > gpurun_out/gab/g_q$q.json 2> gpurun_out/gab/g_q$q.err || exit 1
echo "graphs q=$q $(cat gpurun_out/gab/g_q$q.json)"
timeout -k 10 200 python -u bench_serve.py qps --qps $q --duration 10 --no-graphs > gpurun_out/gab/e_q$q.json 2> gpurun_out/gab/e_q$q.err || exit 1
echo "eager q=$q $(cat gpurun_out/gab/e_q$q.json)"
done
