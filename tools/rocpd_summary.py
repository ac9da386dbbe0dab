"""Summarise a rocprofv3 SQLite output (``-d DIR -o run`` -> run_results.db):
per-kernel calls / total / mean time and a per-category breakdown.

    python tools/rocpd_summary.py gpurun_out/prof11/run_results.db [last_ms] > profiles/x.md

``last_ms``: only kernels that start in the last ``last_ms`` milliseconds of
the trace (e.g. the timed steps of bench.py, after model init and warm-up).
"""
import os
import re
import sqlite3
import sys
from collections import defaultdict

CATS = [("gemm (MFMA 256x256, AGPR 1 wave/SIMD)", r"gemm_tn_256d"),
        ("gemm (MFMA 256x256)", r"gemm_tn_256"), ("gemm (MFMA 128x128)", r"gemm_tn_128"),
        ("gemm (flex tiles)", r"gemm_tn_flex"), ("gemm (hipBLASLt, plan 'lib' buckets)", r"Cijk_"),
        ("gemm (skinny K2)", r"gemm_skinny"), ("gemm (K2 weight-streaming)", r"gemm_stream|stream_"),
        ("split-K reduce", r"splitk_reduce"), ("attention", r"attn_"),
        ("sampling", r"sample_"), ("rmsnorm", r"rmsnorm"), ("rope+kv write", r"rope"),
        ("embedding", r"embedding"), ("top-k", r"topk|l2norm"), ("kv copy", r"copy_blocks"),
        ("all-reduce", r"car_|nccl|rccl"), ("torch/other", r".")]


def short(name):
    if os.environ.get("MCP_SUMMARY_FULL_NAMES") == "1":   # e.g. hipBLASLt's tile / split fields
        return name
    n = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", name)
    m = re.match(r"(\w+?)I(.*)E(vPK|v)", n)
    return (m.group(1) + "<" + m.group(2)[:40] + ">") if m else n[:80]


def main(db, last_ms=None):
    c = sqlite3.connect(db)
    t_end = c.execute("select max(end) from kernels").fetchone()[0]
    t0 = t_end - int(last_ms * 1e6) if last_ms else 0
    rows = list(c.execute("select name, count(*), sum(duration), avg(duration) from kernels "
                          "where start >= ? group by name order by sum(duration) desc", (t0,)))
    span = c.execute("select max(end) - min(start) from kernels where start >= ?",
                     (t0,)).fetchone()[0]
    total = sum(r[2] for r in rows)
    cats = defaultdict(float)
    for name, n, tot, avg in rows:
        for cat, pat in CATS:
            if re.search(pat, name):
                cats[cat] += tot
                break
    print(f"# rocprofv3 kernel summary: `{db}`\n")
    print(f"GPU kernel time {total / 1e6:.1f} ms over a {span / 1e6:.1f} ms window "
          f"(busy {100 * total / span:.1f} %)\n")
    print("| category | ms | % of kernel time |\n|---|---|---|")
    for cat, _ in CATS:
        if cats.get(cat):
            print(f"| {cat} | {cats[cat] / 1e6:.1f} | {100 * cats[cat] / total:.1f} |")
    print("\n| kernel | calls | total ms | mean us | % |\n|---|---|---|---|---|")
    for name, n, tot, avg in rows[:25]:
        print(f"| `{short(name)}` | {n} | {tot / 1e6:.2f} | {avg / 1e3:.1f} | {100 * tot / total:.1f} |")
    other = [r for r in rows if not any(re.search(p, r[0]) for _, p in CATS[:-1])]
    if other:
        print("\n| uncategorised kernel | calls | total ms | mean us |\n|---|---|---|---|")
        for name, n, tot, avg in other[:12]:
            print(f"| `{name[:110]}` | {n} | {tot / 1e6:.2f} | {avg / 1e3:.1f} |")
    # idle time between kernels (union of kernel intervals on the device):
    # host-side gaps (scheduling, grammar, H2D, first launch) show up as the
    # long ones; launch-to-launch bubbles as the short ones
    iv = sorted(c.execute("select start, end from kernels where start >= ?", (t0,)))
    gaps, cur = [], None
    for s, e in iv:
        if cur is not None and s > cur:
            gaps.append(s - cur)
        cur = e if cur is None else max(cur, e)
    edges = [(0, 10e3), (10e3, 100e3), (100e3, 1e6), (1e6, 1e12)]
    labels = ["< 10 us", "10-100 us", "0.1-1 ms", "> 1 ms"]
    print("\n| idle gap | count | total ms | % of window |\n|---|---|---|---|")
    for (lo, hi), lab in zip(edges, labels):
        g = [x for x in gaps if lo <= x < hi]
        print(f"| {lab} | {len(g)} | {sum(g) / 1e6:.1f} | {100 * sum(g) / span:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else None)
