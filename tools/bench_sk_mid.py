"""Whole-launch stream-K vs the planned path at mid M (one wave of 256-row or
192-row tiles that leaves CUs idle: N = 4096 shapes at M = 2048-4096, qkv just
past a wave boundary).  Cold weights, epilogue 0 for every candidate (the
tuning entry points), torch.matmul (hipBLASLt) for reference.

    python tools/bench_sk_mid.py [m0 m1 step]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402

L = ops.lib()
m0, m1, mstep = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (2048, 4096, 128)
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


for (N, K) in [(4096, 14336), (4096, 4096), (6144, 4096), (28672, 4096)]:
    X = torch.randn(m1, K, device=dev).bfloat16()
    Y = torch.empty(m1, N, device=dev, dtype=torch.bfloat16)
    Ws = [(torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
          for _ in range(max(2, int(1.2e9 // (N * K * 2))))]
    for M in range(m0, m1 + 1, mstep):
        x, y = X[:M], Y[:M]
        ref = (x[:64].float() @ Ws[0].float().t())
        L.gemm_variant(x, Ws[0], y, 50)
        err = ((y[:64].float() - ref).norm() / ref.norm()).item()
        row = {"N": N, "K": K, "M": M, "sk_err": round(err, 5)}
        for name, fn in (("plan", lambda i: ops.gemm(x, Ws[i], out=y)),
                         ("sk", lambda i: L.gemm_variant(x, Ws[i], y, 50)),
                         ("agpr256", lambda i: L.gemm_variant(x, Ws[i], y, 49)),
                         ("agpr192", lambda i: L.gemm_variant(x, Ws[i], y, 51)),
                         ("torch", lambda i: torch.matmul(x, Ws[i].t()))):
            row[name] = round(time_us(fn, len(Ws)), 1)
        print(json.dumps(row), flush=True)
    del X, Y, Ws
