"""A/B of GEMM dispatch knobs over the headline's own GEMM mix, interleaved in
one process (cdna_hip_programming.md §5.4 rule 24), cold weights (each call
reads the next of > 1 GB of weight copies), production epilogues.

    python tools/bench_gemm_ab.py ARM_A ARM_B [--trace F] [--min-m 256] [--rounds 3]

An arm is a comma list of ``force_fn=value`` on ``ops.lib()`` (e.g.
``gemm_wide_force=0`` vs ``gemm_wide_force=1,gemm_persist_force=1``).  Per
(N, K, M) of the trace (calls >= 1, M >= min-m): the min over rounds of each
arm's mean time, the call-weighted family totals, and the largest output
difference between the arms (both against an fp32 reference on one call).
"""
import argparse
import collections
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402
from mcp_amd.ops import reference as refops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("a")
ap.add_argument("b")
ap.add_argument("--trace", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                 "bench_data", "gemm_trace_bench_r4.jsonl"))
ap.add_argument("--min-m", type=int, default=256)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--ms", default="", help="only these M (comma list)")
args = ap.parse_args()


def arm(spec):
    out = []
    for kv in filter(None, spec.split(",")):
        k, v = kv.split("=")
        out.append((getattr(ops.lib(), k), int(v)))
    return out


ARMS = {"a": arm(args.a), "b": arm(args.b)}


def apply(name):
    for fn, v in ARMS[name]:
        fn(v)


calls = collections.Counter()
for line in open(args.trace):
    if line.startswith("{"):
        r = json.loads(line)
        if r["M"] >= args.min_m:
            calls[(r["N"], r["K"], r["M"])] += r["calls"]
only = {int(x) for x in args.ms.split(",") if x}
dev = "cuda"
s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def time_us(fn, n, reps=6):
    fn(0)
    s_ev.record()
    for i in range(reps):
        fn(i % n)
    e_ev.record()
    torch.cuda.synchronize()
    return s_ev.elapsed_time(e_ev) * 1e3 / reps


KIND = {(4096, 4096): "o+res", (28672, 4096): "gate|up", (4096, 14336): "down+res",
        (6144, 4096): "qkv"}
tot = collections.defaultdict(lambda: [0.0, 0.0, 0.0])
worst = 0.0
for (N, K), fam in KIND.items():
    ms = sorted(M for (n, k, M) in calls if (n, k) == (N, K) and (not only or M in only))
    if not ms:
        continue
    mmax = max(ms)
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(mmax, K, device=dev, generator=g).bfloat16()
    R = torch.randn(mmax, N // 2 if fam == "gate|up" else N, device=dev, generator=g).bfloat16()
    Ws = [(torch.randn(N, K, device=dev, generator=g) / K ** 0.5).bfloat16()
          for _ in range(max(2, int(1.2e9 // (N * K * 2))))]
    for M in ms:
        x, r = X[:M], R[:M]
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        if fam == "gate|up":
            fn = lambda i: ops.gemm_silu(x, Ws[i])
        elif fam == "qkv":
            fn = lambda i: ops.gemm(x, Ws[i], out=y)
        else:
            fn = lambda i: ops.gemm(x, Ws[i], R=r, out=y)
        outs = {}
        for a in ("a", "b"):
            apply(a)
            o = fn(0)
            outs[a] = (o if o is not None else y).float().clone()
        if fam == "gate|up":
            ref = refops.gemm_silu(x, Ws[0]).float()
        else:
            ref = x.float() @ Ws[0].float().t()
            if fam != "qkv":
                ref = ref + r.float()
        errs = {a: float((outs[a] - ref).abs().max() / ref.abs().max()) for a in outs}
        diff = float((outs["a"] - outs["b"]).abs().max())
        worst = max(worst, errs["a"], errs["b"])
        best = {"a": float("inf"), "b": float("inf")}
        for _ in range(args.rounds):
            for a in ("a", "b"):
                apply(a)
                best[a] = min(best[a], time_us(fn, len(Ws)))
        c = calls[(N, K, M)]
        t = tot[fam]
        t[0] += 2 * M * N * K * c
        t[1] += best["a"] * c
        t[2] += best["b"] * c
        print(json.dumps({"N": N, "K": K, "M": M, "calls": c, "a_us": round(best["a"], 1),
                          "b_us": round(best["b"], 1), "b_over_a": round(best["a"] / best["b"], 4),
                          "rel_err": {k: round(v, 5) for k, v in errs.items()},
                          "a_vs_b_maxdiff": diff}), flush=True)
    del X, R, Ws
for fam, (f, a, b) in tot.items():
    print(json.dumps({"family": fam, "a_tf": round(f / a / 1e6, 1), "b_tf": round(f / b / 1e6, 1),
                      "a_ms": round(a / 1e3, 2), "b_ms": round(b / 1e3, 2),
                      "speedup_b": round(a / b, 4)}), flush=True)
fa = sum(v[1] for v in tot.values())
fb = sum(v[2] for v in tot.values())
print(json.dumps({"total_a_ms": round(fa / 1e3, 2), "total_b_ms": round(fb / 1e3, 2),
                  "speedup_b": round(fa / fb, 4), "worst_rel_err": round(worst, 5),
                  "arms": [args.a, args.b]}), flush=True)
