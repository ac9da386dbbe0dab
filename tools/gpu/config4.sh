set -o pipefail
mkdir -p gpurun_out/c4
export TMPDIR=/tmp
timeout -k 10 900 python -u bench_tp.py --steps 3 --warmup 1 > gpurun_out/c4/c4.json 2> gpurun_out/c4/c4.err || { tail -20 gpurun_out/c4/c4.err; exit 1; }
cat gpurun_out/c4/c4.json; tail -5 gpurun_out/c4/c4.err
