"""Cold-weight timing of the mid-M (48-256 token) projections config 5 runs:
the shipped dispatch (measured plan) against the weight-streaming kernel at
forced split counts (it serves M <= 128).
    python tools/bench_midm_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402

L = ops.lib()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def t_us(fn, R, n=24):
    for i in range(R):
        fn(i)
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(3):
        e0.record()
        for i in range(n):
            fn(i % R)
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / n * 1e3)
    return round(best, 1)


for (N, K, kind) in [(4096, 14336, "res"), (6144, 4096, "plain"), (4096, 4096, "res"),
                     (28672, 4096, "swiglu")]:
    R = max(4, int(1.6e9 // (N * K * 2)) + 1)
    Ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(R)]
    for M in (48, 64, 96, 128, 192, 256):
        X = torch.randn(M, K, device="cuda").bfloat16()
        Y = torch.empty(M, N // 2 if kind == "swiglu" else N, device="cuda", dtype=torch.bfloat16)
        Rr = torch.randn(M, N, device="cuda").bfloat16() if kind == "res" else None
        r = {"M": M, "N": N, "K": K, "kind": kind, "floor_us": round(N * K * 2 / 6.0e12 * 1e6, 1)}
        if kind == "swiglu":
            r["auto_us"] = t_us(lambda i: L.gemm_silu(X, Ws[i], Y, None, 0.0), R)
        else:
            r["auto_us"] = t_us(lambda i: L.gemm(X, Ws[i], Y, Rr, -1), R)
            if M <= 128:
                for S in (1, 2, 4, 8):
                    L.gemm_stream_force_splits(S)
                    r[f"stream_s{S}_us"] = t_us(lambda i: L.gemm(X, Ws[i], Y, Rr, 3), R)
                L.gemm_stream_force_splits(0)
        print(json.dumps(r), flush=True)
    del Ws
