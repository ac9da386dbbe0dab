set -o pipefail
mkdir -p gpurun_out/flex
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/bench_flex.py > gpurun_out/flex/cold.jsonl 2> gpurun_out/flex/err.txt || { tail -20 gpurun_out/flex/err.txt; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/flex/cold.jsonl'):
    d=json.loads(l); print(d['M'], d['N'], d['K'], 'auto', d['auto_us'], 'best', d['best_flex'], 'torch', d['torch_us'])
"
