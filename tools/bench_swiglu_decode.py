"""Cold-weight timing of the decode-sized SwiGLU (gate|up) GEMM: the skinny
kernel's two forms (8 gate + 8 up rows per block vs 32-row blocks) and the
weight-streaming kernel at its split counts.
    python tools/bench_swiglu_decode.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402

L = ops.lib()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def t_us(fn, R, n=28):
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


# gemm_silu dispatch at these M: skinny kernel first for M <= 8 (wide N), the
# weight-streaming kernel for 9..32 (gemm.hip skinny_first / gemm_stream_pick)
for (N, K) in [(28672, 4096), (14336, 4096), (57344, 8192)]:
    R = max(4, int(1.6e9 // (N * K * 2)) + 1)
    Ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(R)]
    for M in (1, 4, 8, 12, 16):
        X = torch.randn(M, K, device="cuda").bfloat16()
        Y = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
        r = {"M": M, "N": N, "K": K, "floor_us": round(N * K * 2 / 6.0e12 * 1e6, 1)}
        for h in (2, 0):
            L.gemm_skinny_half(h)
            r[f"half{h}_us"] = t_us(lambda i: L.gemm_silu(X, Ws[i], Y, None, 0.0), R)
        L.gemm_skinny_half(1)
        print(json.dumps(r), flush=True)
    del Ws
