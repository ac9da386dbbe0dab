"""Attribute the device's idle gaps to host phases: reads a rocprofv3
``--kernel-trace --marker-trace`` SQLite output (bench run with MCP_ROCTX=1),
finds every gap between kernels longer than ``min_us`` in the last
``last_ms`` of the trace, and sums, per roctx range name, the part of the
gaps that range covers (a gap can be covered by nested ranges: each is
counted).  Also prints the schema of the marker table it used.

    python tools/gap_attribution.py run_results.db [last_ms] [min_us]
"""
import sqlite3
import sys
from collections import defaultdict


def main(db, last_ms=None, min_us=200.0):
    c = sqlite3.connect(db)
    objs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
    t_end = c.execute("select max(end) from kernels").fetchone()[0]
    t0 = t_end - int(last_ms * 1e6) if last_ms else 0
    iv = sorted(c.execute("select start, end from kernels where start >= ?", (t0,)))
    gaps, cur = [], None
    for s, e in iv:
        if cur is not None and s - cur > min_us * 1e3:
            gaps.append((cur, s))
        cur = e if cur is None else max(cur, e)
    span = iv[-1][1] - iv[0][0]
    # marker ranges: the first table / view with name + start + end besides kernels
    rng = []
    used = None
    for o in objs:
        if o in ("kernels",) or "kernel" in o.lower():
            continue
        try:
            cols = [r[1] for r in c.execute(f"pragma table_info('{o}')")]
        except sqlite3.Error:
            continue
        if {"start", "end"} <= set(cols) and ("name" in cols or "message" in cols):
            nm = "name" if "name" in cols else "message"
            rows = list(c.execute(f"select {nm}, start, end from '{o}' where end >= ?", (t0,)))
            if rows and any(isinstance(r[0], str) and "." in r[0] for r in rows):
                rng, used = rows, (o, cols)
                break
    print(f"# device idle gaps > {min_us:.0f} us: {len(gaps)} gaps, "
          f"{sum(b - a for a, b in gaps) / 1e6:.1f} ms of a {span / 1e6:.1f} ms window\n")
    print(f"marker table: {used}\n")
    if used is None:                       # show the schema to pick the right table next time
        for o in objs:
            try:
                cols = [r[1] for r in c.execute(f"pragma table_info('{o}')")]
            except sqlite3.Error:
                cols = []
            print(f"- `{o}`: {', '.join(cols)}")
    cover = defaultdict(float)
    for a, b in gaps:
        for name, s, e in rng:
            lo, hi = max(a, s), min(b, e)
            if hi > lo:
                cover[name] += hi - lo
    print("| host range | ms of gap covered | per gap us |\n|---|---|---|")
    for name, t in sorted(cover.items(), key=lambda x: -x[1]):
        print(f"| `{name}` | {t / 1e6:.1f} | {t / 1e3 / max(1, len(gaps)):.0f} |")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else None,
         float(sys.argv[3]) if len(sys.argv) > 3 else 200.0)
