"""Replay the headline bench's GEMM mix (profiles/gemm_shapes_bench_r1.jsonl:
every (M, N, K) the bench launched, with its call count) through our
dispatch - with the production epilogue of each projection - and through
hipBLASLt (torch), cold weights (each call reads the next of > 1 GB of weight
copies, as a decode step streams the whole model).  Prints per-shape-family
totals weighted by the calls, so the efficiency of each family at the bench's
own sizes is measured rather than inferred from single sizes.

    python tools/bench_gemm_mix.py [trace.jsonl] [min_M]
"""
import collections
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402

trace = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "gemm_shapes_bench_r1.jsonl")
min_m = int(sys.argv[2]) if len(sys.argv) > 2 else 256
rows = [json.loads(l) for l in open(trace) if l.startswith("{")]
calls = collections.Counter()
for r in rows:
    if r["M"] >= min_m:
        calls[(r["N"], r["K"], r["M"])] += r["calls"]

dev = "cuda"
s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def time_us(fn, n, reps=6):
    fn(0)
    best = float("inf")
    for _ in range(3):
        s_ev.record()
        for i in range(reps):
            fn(i % n)
        e_ev.record()
        torch.cuda.synchronize()
        best = min(best, s_ev.elapsed_time(e_ev) * 1e3 / reps)
    return best


KIND = {(6144, 4096): "qkv", (4096, 4096): "o+res", (28672, 4096): "gate|up", (4096, 14336): "down+res"}
tot = collections.defaultdict(lambda: [0.0, 0.0, 0.0])   # family -> [flop, ours us, torch us]
for (N, K) in KIND:
    ms = sorted(M for (n, k, M) in calls if (n, k) == (N, K))
    if not ms:
        continue
    mmax = max(ms)
    X = torch.randn(mmax, K, device=dev).bfloat16()
    R = torch.randn(mmax, N, device=dev).bfloat16()
    Ws = [(torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
          for _ in range(max(2, int(1.2e9 // (N * K * 2))))]
    fam = KIND[(N, K)]
    for M in ms:
        x, r = X[:M], R[:M]
        if fam == "gate|up":
            ours = lambda i: ops.gemm_silu(x, Ws[i])                       # SwiGLU epilogue
            lib = lambda i: torch.matmul(x, Ws[i].t())                    # GEMM alone
        elif fam == "qkv":
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            ours = lambda i: ops.gemm(x, Ws[i], out=y)
            lib = lambda i: torch.matmul(x, Ws[i].t())
        else:
            y = r.clone()
            ours = lambda i: ops.gemm(x, Ws[i], R=y, out=y)               # residual epilogue
            lib = lambda i: torch.addmm(r, x, Ws[i].t())                  # beta = 1 epilogue
        a, b = time_us(ours, len(Ws)), time_us(lib, len(Ws))
        c = calls[(N, K, M)]
        f = 2 * M * N * K
        t = tot[fam]
        t[0] += f * c
        t[1] += a * c
        t[2] += b * c
        print(json.dumps({"N": N, "K": K, "M": M, "calls": c, "ours_us": round(a, 1),
                          "torch_us": round(b, 1), "ours_tf": round(f / a / 1e6, 1),
                          "torch_tf": round(f / b / 1e6, 1),
                          "select": ops.lib().gemm_select(M, N, K)}), flush=True)
    del X, R, Ws
for fam, (f, a, b) in tot.items():
    print(json.dumps({"family": fam, "flop_weighted_ours_tf": round(f / a / 1e6, 1),
                      "flop_weighted_torch_tf": round(f / b / 1e6, 1),
                      "ours_ms": round(a / 1e3, 1), "torch_ms": round(b / 1e3, 1)}), flush=True)
