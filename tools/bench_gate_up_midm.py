"""gate|up + SwiGLU at mid M: the shipped dispatch, every
AGPR height with the whole K (plan codes 1-5) and with K halves over two
workgroups per tile (codes 401-405, gemm256d.hip SPLIT 2), against hipBLASLt
(torch.matmul: the plain GEMM alone, and + the separate silu_mul the fused
epilogue saves).  Llama-3-8B gate|up: N = 28672 (interleaved), K = 4096.
Cold weights (a rotation of copies larger than the 256 MB Infinity Cache),
synthetic data, best of 3 x 12 launches.

    python tools/bench_gate_up_midm.py [M ...]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402

L = ops.lib()
N, K = 28672, 4096
Ms = [int(a) for a in sys.argv[1:]] or [129, 160, 192, 224, 256, 288, 320, 384]
R = 6                                                   # 6 x 235 MB > the MALL
Ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(R)]
WTs = [w.t() for w in Ws]
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def t_us(fn, n=12):
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


for M in Ms:
    X = torch.randn(M, K, device="cuda").bfloat16()
    Y = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
    P = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    rec = {"M": M, "N": N, "K": K}
    rec["dispatch_us"] = t_us(lambda i: L.gemm_silu(X, Ws[i], Y, None, 0.0))
    for code in (1, 2, 3, 4, 5, 401, 402, 403, 404, 405):
        if L.gemm_silu_algo(X, Ws[0], Y, code, None, 0.0) == 0:
            rec[f"code{code}_us"] = t_us(lambda i, c=code: L.gemm_silu_algo(X, Ws[i], Y, c, None, 0.0))
    L.gemm_pf_force(1)                                  # the split form + W L2 fills
    for code in (401, 402, 403, 404, 405):
        if L.gemm_silu_algo(X, Ws[0], Y, code, None, 0.0) == 0:
            rec[f"code{code}pf_us"] = t_us(lambda i, c=code: L.gemm_silu_algo(X, Ws[i], Y, c, None, 0.0))
    L.gemm_pf_force(-1)
    rec["hipblaslt_gemm_us"] = t_us(lambda i: torch.matmul(X, WTs[i], out=P))
    rec["hipblaslt_gemm_silu_us"] = t_us(lambda i: (torch.matmul(X, WTs[i], out=P), L.silu_mul(P, Y)))
    ours = min(v for k, v in rec.items() if k.startswith("code") or k == "dispatch_us")
    rec["best_ours_us"] = ours
    rec["best_ours_tflops"] = round(2 * M * N * K / ours / 1e6, 1)
    print(json.dumps(rec), flush=True)
