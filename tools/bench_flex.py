"""Serving-size GEMMs: the auto path vs every flex tile (gemm_flex.hip) vs
torch.matmul (hipBLASLt), COLD weights (each call takes the next of R weight
copies, > 1.5 GB in all, so nothing is served from the 256 MB Infinity Cache -
a serving step streams the whole model).  Checks every flex result against an
fp32 reference once.
    python tools/bench_flex.py [M,M,...] [--warm]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402

L = ops.lib()
args = [a for a in sys.argv[1:] if not a.startswith("--")]
warm = "--warm" in sys.argv
Ms = [int(x) for x in args[0].split(",")] if args else [256, 384, 512, 640, 768, 1024, 1536, 2048]
SHAPES = [(6144, 4096, False), (4096, 4096, True), (4096, 14336, True)]
NC = L.gemm_flex_count()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def t_us(fn, R, n=24):
    for i in range(min(R, 4)):
        fn(i)
    torch.cuda.synchronize()
    e0.record()
    for i in range(n):
        fn(i % R)
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / n * 1e3, 1)


for N, K, res in SHAPES:
    R = 1 if warm else max(2, int(1.5e9 // (N * K * 2)) + 1)
    Ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(R)]
    for M in Ms:
        X = torch.randn(M, K, device="cuda").bfloat16()
        Rr = torch.randn(M, N, device="cuda").bfloat16() if res else None
        Y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ref = X.float() @ Ws[0].float().t() + (Rr.float() if res else 0)
        row = {"M": M, "N": N, "K": K, "res": res, "cold": not warm}
        row["auto_us"] = t_us(lambda i: L.gemm(X, Ws[i], Y, Rr, -1), R)
        best = None
        for c in list(range(NC)) + [32 + c for c in range(NC)]:   # 2-stage, 4-stage
            L.gemm(X, Ws[0], Y, Rr, 16 + c)
            err = ((Y.float() - ref).norm() / ref.norm()).item()
            assert err < 1e-2, (M, N, K, c, err)
            us = t_us(lambda i: L.gemm(X, Ws[i], Y, Rr, 16 + c), R)
            row[f"f{c}"] = us
            if best is None or us < best[1]:
                best = (c, us)
        row["best_flex"] = best
        if res:
            row["torch_us"] = t_us(lambda i: torch.addmm(Rr, X, Ws[i].t()), R)
        else:
            row["torch_us"] = t_us(lambda i: torch.matmul(X, Ws[i].t()), R)
        print(json.dumps(row), flush=True)
