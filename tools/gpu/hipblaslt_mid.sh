set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hbl
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/hbl/db -o run --output-format csv -- python3 tools/gpu/hipblaslt_mid.py > gpurun_out/hbl/log.txt 2>&1 || { tail -20 gpurun_out/hbl/log.txt; exit 1; }
f=$(find gpurun_out/hbl/db -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
seen = []
for r in rows:
    n = r.get('Kernel_Name', '')
    if 'Cijk' in n or 'gemm' in n.lower():
        g = (n[:160], r.get('Grid_Size_X', r.get('Grid_Size', '')), r.get('Workgroup_Size_X', ''))
        dur = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
        print(g, dur)
PY
rm -rf gpurun_out/hbl/db
