"""Average rocprofv3 --pmc counters per kernel (name filter) from a rocpd db.

    python tools/pmc_summary.py gpurun_out/pmc/v25/run_results.db gemm_tn
    python tools/pmc_summary.py --by-kernel run_results.db     (per-kernel table)
Prints counters averaged over matching dispatches, plus derived clock (GHz)
and MFMA-busy fraction (MI355X_MICROARCH.md: SQ_* cycle counters are
quad-cycles except SQ_VALU_MFMA_BUSY_CYCLES; GRBM_GUI_ACTIVE sums 8 XCDs).
"""
import sqlite3
import sys
from collections import defaultdict


def summarise(db, pat):
    c = sqlite3.connect(db)
    rows = c.execute("select dispatch_id, kernel_name, counter_name, value, duration from "
                     "counters_collection where kernel_name like ?", (f"%{pat}%",)).fetchall()
    per = defaultdict(dict)
    dur = {}
    for d, _, cn, v, du in rows:
        per[d][cn] = per[d].get(cn, 0.0) + v
        dur[d] = du
    if not per:
        return None
    keys = sorted({k for p in per.values() for k in p})
    avg = {k: sum(p.get(k, 0.0) for p in per.values()) / len(per) for k in keys}
    avg["duration_us"] = sum(dur.values()) / len(dur) / 1e3
    if "GRBM_GUI_ACTIVE" in avg:
        avg["clock_GHz"] = avg["GRBM_GUI_ACTIVE"] / 8 / (avg["duration_us"] * 1e3)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
        # per-SIMD MFMA busy over the kernel's active cycles (256 CUs x 4 SIMDs)
        avg["mfma_busy_frac"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * avg["GRBM_GUI_ACTIVE"] / 8)
    return len(per), avg


def by_kernel(db, top=16):
    """Markdown table: every counter summed per kernel (template name), per call."""
    c = sqlite3.connect(db)
    rows = c.execute("select dispatch_id, kernel_name, counter_name, value, duration from "
                     "counters_collection").fetchall()
    per, name, dur = defaultdict(dict), {}, {}
    for d, k, cn, v, du in rows:
        per[d][cn] = per[d].get(cn, 0.0) + v
        name[d], dur[d] = k, du
    keys = sorted({k for p in per.values() for k in p})
    agg = defaultdict(lambda: [0, 0.0, defaultdict(float)])
    for d, p in per.items():
        k = name[d].replace("void ", "").replace("(anonymous namespace)::", "")
        k = (k[:k.index("(")] if "(" in k else k)[:60]
        a = agg[k]
        a[0] += 1
        a[1] += dur[d]
        for cn, v in p.items():
            a[2][cn] += v
    print("| kernel | calls | us / call | " + " | ".join(keys) + " |")
    print("|---|---|---|" + "---|" * len(keys))
    for k, (n, du, cs) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
        print(f"| `{k}` | {n} | {du / n / 1e3:.1f} | " + " | ".join(f"{cs[c] / n:.4g}" for c in keys) + " |")


if __name__ == "__main__":
    if sys.argv[1] == "--by-kernel":
        by_kernel(sys.argv[2])
        sys.exit(0)
    for db in sys.argv[1:-1]:
        r = summarise(db, sys.argv[-1])
        if r is None:
            print(db, "no matching dispatches")
            continue
        n, avg = r
        print(f"{db}  ({n} dispatches)")
        for k, v in avg.items():
            print(f"   {k:28s} {v:.4g}")
