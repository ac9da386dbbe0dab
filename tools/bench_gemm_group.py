"""Tile-group sweep of the AGPR GEMM (gemm256d.hip) with cold weights: for
the Llama-3-8B projections at the headline's step sizes, time the production
dispatch (plan height, production epilogue) with the grouped tile order at
``group`` M-tiles per W panel, interleaved rounds in one process, each call
on the next of > 1.5 GB of weight copies (a serving step streams the model).

    python tools/bench_gemm_group.py [out.jsonl] [M,M,...] [g,g,...]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else None
MS = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1536, 2048, 2560, 3072, 3584, 4096]
GS = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 2, 4, 8, 16, 64]
L = ops.lib()
dev = "cuda"
s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
SHAPES = [("qkv", 6144, 4096), ("o+res", 4096, 4096), ("gate|up", 28672, 4096), ("down+res", 4096, 14336)]


def time_us(fn, n, reps=8):
    fn(0)
    s_ev.record()
    for i in range(reps):
        fn(1 + i % (n - 1))
    e_ev.record()
    torch.cuda.synchronize()
    return s_ev.elapsed_time(e_ev) * 1e3 / reps


for fam, N, K in SHAPES:
    mmax = max(MS)
    X = torch.randn(mmax, K, device=dev).bfloat16()
    R = torch.randn(mmax, N, device=dev).bfloat16()
    Ws = [(torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
          for _ in range(max(3, int(1.6e9 // (N * K * 2))))]
    for M in MS:
        x = X[:M]
        if L.gemm_select(M, N, K) != 1:
            continue
        if fam == "gate|up":
            y = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
            fn = lambda i: ops.gemm_silu(x, Ws[i], out=y)
        elif fam == "qkv":
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            fn = lambda i: ops.gemm(x, Ws[i], out=y)
        else:
            y = R[:M].clone()
            fn = lambda i: ops.gemm(x, Ws[i], R=y, out=y)
        best = {g: float("inf") for g in GS}
        for _ in range(3):
            for g in GS:
                L.gemm_group_force(g)
                best[g] = min(best[g], time_us(fn, len(Ws)))
        L.gemm_group_force(0)
        f = 2 * M * N * K
        rec = {"family": fam, "N": N, "K": K, "M": M, "height": L.gemm_plan_lookup(M, N, K),
               "us": {str(g): round(v, 1) for g, v in best.items()},
               "tflops": {str(g): round(f / v / 1e6, 1) for g, v in best.items()},
               "best_group": min(best, key=best.get),
               "gain_vs_4": round(best[4] / min(best.values()), 3) if 4 in best else None}
        print(json.dumps(rec), flush=True)
        if out:
            with open(out, "a") as fh:
                fh.write(json.dumps(rec) + "\n")
    del X, R, Ws
    torch.cuda.empty_cache()
