"""Cold-weight (HBM-streamed) sweep of the K2 weight-streaming kernel's split
count against the skinny kernel, for the tiny-M steps of a single intent.
    python tools/bench_cold_stream.py"""
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
    e0.record()
    for i in range(n):
        fn(i % R)
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / n * 1e3, 1)


for (N, K) in [(28672, 4096), (4096, 14336), (6144, 4096), (4096, 4096)]:
    R = max(4, int(1.6e9 // (N * K * 2)) + 1)
    Ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(R)]
    for M in (1, 4, 8, 12, 16, 24, 32):
        X = torch.randn(M, K, device="cuda").bfloat16()
        Y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        r = {"M": M, "N": N, "K": K, "floor_us": round(N * K * 2 / 6.0e12 * 1e6, 1)}
        r["skinny_us"] = t_us(lambda i: L.gemm(X, Ws[i], Y, None, 2), R)
        r["auto_us"] = t_us(lambda i: L.gemm(X, Ws[i], Y, None, -1), R)
        for S in (1, 2, 3, 4, 8):
            L.gemm_stream_force_splits(S)
            r[f"stream_s{S}_us"] = t_us(lambda i: L.gemm(X, Ws[i], Y, None, 3), R)
        L.gemm_stream_force_splits(0)
        print(json.dumps(r), flush=True)
    del Ws
