"""Fused split-K sweep of the 128^2 kernel at the Llama-3-8B projection shapes:
every admissible split count S (gemm_splitk_force) per (M, N, K), plus the
production choice (auto) and torch.matmul (hipBLASLt).  One JSON line per
(shape, M): times in us, the best S, and weight bytes/s of the best.
    python tools/bench_splitk.py [M,M,...]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402

L = ops.lib()
Ms = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else \
    [16, 32, 64, 96, 128, 192, 256, 320, 384, 448, 512]
SHAPES = [(6144, 4096, 0), (4096, 4096, 1), (28672, 4096, 2), (4096, 14336, 1)]
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def t_us(fn, n=20):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / n * 1e3)
    return round(best, 1)


for (N, K, epi) in SHAPES:
    W = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    for M in Ms:
        X = torch.randn(M, K, device="cuda").bfloat16()
        R = torch.randn(M, N, device="cuda").bfloat16()
        Y = torch.empty(M, N // 2 if epi == 2 else N, device="cuda", dtype=torch.bfloat16)
        if epi == 2:
            fn = lambda: L.gemm_silu(X, W, Y)  # noqa: E731
        elif epi == 1:
            fn = lambda: L.gemm(X, W, Y, R, 0)  # noqa: E731
        else:
            fn = lambda: L.gemm(X, W, Y, None, 0)  # noqa: E731
        r = {"M": M, "N": N, "K": K, "epi": epi}
        for S in [1, 2, 3, 4, 6, 8, 12, 16, 32]:
            L.gemm_splitk_force(S)
            if S > 1 and L.gemm128_splits(M, N, K) != S:
                continue
            r[f"S{S}"] = t_us(fn)
        L.gemm_splitk_force(-1)
        if M <= 128:                       # K2 stream kernel (algo 3 / SwiGLU entry)
            for S in [0, 1, 2, 4, 8]:
                L.gemm_stream_force_splits(S)
                if epi == 2:
                    f2 = lambda: L.gemm_silu(X, W, Y)  # noqa: E731
                else:
                    f2 = lambda: L.gemm(X, W, Y, R if epi else None, 3)  # noqa: E731
                r[f"st{S}"] = t_us(f2)
            L.gemm_stream_force_splits(0)
            r["st_auto_S"] = L.gemm_stream_splits(M, N, K, epi)
            L.gemm_stream_force_splits(0)
        r["auto_S"] = L.gemm128_splits(M, N, K)
        r["auto"] = t_us(lambda: (L.gemm_silu(X, W, Y) if epi == 2 else L.gemm(X, W, Y, R if epi else None, -1)))
        r["torch"] = t_us(lambda: torch.matmul(X, W.t()))
        best = min((v, k) for k, v in r.items() if k.startswith("S") or (k.startswith("st") and k[2:].isdigit()))
        r["best"], r["best_us"] = best[1], best[0]
        r["TBps_best"] = round(N * K * 2 / best[0] / 1e6, 2)
        r["TBps_auto"] = round(N * K * 2 / r["auto"] / 1e6, 2)
        print(json.dumps(r), flush=True)
