set -o pipefail
mkdir -p gpurun_out/nt128
export TMPDIR=/tmp
MCP_GEMM128_NT_MAXM=1024 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" > gpurun_out/nt128/tests.log 2>&1 || { tail -30 gpurun_out/nt128/tests.log; exit 1; }
tail -2 gpurun_out/nt128/tests.log
for nt in 0 1024 0 1024; do
  MCP_GEMM128_NT_MAXM=$nt timeout -k 10 300 python -u tools/bench_cold_small_m.py 64,128,256,384,512,768 > gpurun_out/nt128/c_$nt.jsonl 2>gpurun_out/nt128/err.txt || { tail -5 gpurun_out/nt128/err.txt; exit 1; }
  echo "nt=$nt"; python3 -c "
import json
for l in open('gpurun_out/nt128/c_$nt.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d['M'], d['N'], d['K'], d.get('auto_us'), d.get('128_us'), d.get('swiglu_auto_us',''), d.get('torch_us'))
"
done
