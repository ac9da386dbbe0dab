"""Aligned split-K (gemm256sk.hip: tiles x S workgroups, one k-slice each,
last arriver sums the S slabs) vs our data-parallel grids and hipBLASLt, cold
weights, epilogue 0, on the residual-projection shapes at mid M.

    python tools/bench_sk_split.py [m0 m1 step]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402

L = ops.lib()
m0, m1, mstep = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (1024, 4096, 256)
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


for (N, K) in [(4096, 14336), (4096, 4096)]:
    X = torch.randn(m1, K, device="cuda").bfloat16()
    Y = torch.empty(m1, N, device="cuda", dtype=torch.bfloat16)
    Ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
          for _ in range(max(2, int(1.2e9 // (N * K * 2))))]
    vs = [62, 64, 68] + ([67, 614] if K == 14336 else [])
    for M in range(m0, m1 + 1, mstep):
        x, y = X[:M], Y[:M]
        ref = x.float() @ Ws[0].float().t()
        row = {"N": N, "K": K, "M": M}
        for v in vs:
            L.gemm_variant(x, Ws[0], y, v)
            torch.cuda.synchronize()
            row[f"err{v}"] = round(((y.float() - ref).norm() / ref.norm()).item(), 5)
            row[f"s{v}"] = round(time_us(lambda i: L.gemm_variant(x, Ws[i], y, v), len(Ws)), 1)
        row["dp192"] = round(time_us(lambda i: L.gemm_variant(x, Ws[i], y, 51), len(Ws)), 1)
        row["dp256"] = round(time_us(lambda i: L.gemm_variant(x, Ws[i], y, 49), len(Ws)), 1)
        row["torch"] = round(time_us(lambda i: torch.matmul(x, Ws[i].t()), len(Ws)), 1)
        print(json.dumps(row), flush=True)
    del X, Y, Ws
