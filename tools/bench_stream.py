"""K2 stream-kernel sweep (gemm_stream.hip) at the Llama-3-8B projection
shapes: split counts S (0 = the kernel's own rule) per (M, N, K); one JSON
line per (shape, M) with times in us and weight TB/s of the best.
    MCP_GEMM_STREAM_NT=0|1 python tools/bench_stream.py [M,M,...]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402

L = ops.lib()
Ms = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 16, 32, 64, 96, 128]
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
        fn = (lambda: L.gemm_silu(X, W, Y)) if epi == 2 else (lambda: L.gemm(X, W, Y, R if epi else None, 3))
        r = {"M": M, "N": N, "K": K, "epi": epi, "nt": os.environ.get("MCP_GEMM_STREAM_NT", "0"),
             "auto_S": L.gemm_stream_splits(M, N, K, epi)}
        for S in [0, 1, 2, 4, 8]:
            L.gemm_stream_force_splits(S)
            r[f"S{S}"] = t_us(fn)
        L.gemm_stream_force_splits(0)
        best = min((v, k) for k, v in r.items() if k[0] == "S" and k[1:].isdigit())
        r["best"], r["best_us"] = best[1], best[0]
        r["TBps_best"] = round(N * K * 2 / best[0] / 1e6, 2)
        r["TBps_auto"] = round(N * K * 2 / r["S0"] / 1e6, 2)
        print(json.dumps(r), flush=True)
