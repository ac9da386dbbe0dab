set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ps
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ps -o run -- python3 bench_serve.py single --n 10 > gpurun_out/ps/serve.log 2>&1
python3 tools/rocpd_summary.py gpurun_out/ps/run_results.db 2500 > gpurun_out/ps_summary.md
python3 - <<'PY' > gpurun_out/ps_steps.txt
import sqlite3
c = sqlite3.connect("gpurun_out/ps/run_results.db")
rows = c.execute("select start, end from kernels order by start").fetchall()
t_end = rows[-1][1]
rows = [r for r in rows if r[0] > t_end - 2500e6]
# gaps > 100 us = step boundaries (host round trip)
gaps = []
busy = 0
for a, b in zip(rows, rows[1:]):
    busy += a[1] - a[0]
    g = b[0] - a[1]
    if g > 0: gaps.append(g)
span = rows[-1][1] - rows[0][0]
big = [g for g in gaps if g > 100e3]
print("window_ms", span / 1e6, "kernel_busy_ms", busy / 1e6, "gaps>100us:", len(big), "sum_ms", sum(big) / 1e6,
      "mean_us", (sum(big) / len(big) / 1e3) if big else 0, "small_gaps_sum_ms", sum(g for g in gaps if g <= 100e3) / 1e6)
PY
rm -rf gpurun_out/ps/*.db gpurun_out/ps/*/
