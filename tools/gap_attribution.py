"""Attribute the device's idle gaps to host phases: reads a rocprofv3
``--kernel-trace --marker-trace`` SQLite output (bench run with MCP_ROCTX=1),
finds every gap between kernels longer than ``min_us`` in the last
``last_ms`` of the trace, and sums, per roctx range name, the part of the
gaps that range covers (a gap can be covered by nested ranges: each is
counted).  Also prints the schema of the marker table it used.

    python tools/gap_attribution.py run_results.db [last_ms] [min_us]
"""
import json
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
    if "regions" in objs:                  # rocpd views (rocprofv3 -f rocpd)
        n_all = c.execute("select count(*) from regions").fetchone()[0]
        names = [r[0] for r in c.execute("select distinct name from regions limit 20")]
        print(f"# regions view: {n_all} rows, names {names}")
        rows = list(c.execute("select name, start, end from regions where end >= ?", (t0,)))
        # roctx ranges: the region is the API call (roctxThreadRangeA), the
        # range's text is the "message" of its extdata JSON
        try:
            msg = []
            for ext, s0, e0 in c.execute("select extdata, start, end from regions where end >= ?", (t0,)):
                try:
                    m = json.loads(ext).get("message") if ext else None
                except (ValueError, AttributeError):
                    m = None
                if m:
                    msg.append((m, s0, e0))
            if msg:
                rows = msg
            print(f"# roctx messages: {len(msg)}")
        except sqlite3.Error as e:
            print(f"# extdata read failed: {e}")
        if rows:
            rng, used = rows, ("regions", ["name", "start", "end"])
    for o in ([] if used else objs):
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
    tot, cnt = defaultdict(float), defaultdict(int)
    for name, s0, e0 in rng:
        tot[name] += e0 - s0
        cnt[name] += 1
    print("| host range | ms of gap covered | per gap us | ms in window | calls | us per call |\n|---|---|---|---|---|---|")
    for name, t in sorted(cover.items(), key=lambda x: -x[1]):
        print(f"| `{name}` | {t / 1e6:.1f} | {t / 1e3 / max(1, len(gaps)):.0f} | "
              f"{tot[name] / 1e6:.1f} | {cnt[name]} | {tot[name] / 1e3 / max(1, cnt[name]):.0f} |")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else None,
         float(sys.argv[3]) if len(sys.argv) > 3 else 200.0)
