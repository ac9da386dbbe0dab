"""Persistent vs one-tile-per-workgroup AGPR GEMM (gemm256p.hip vs
gemm256d.hip) with cold weights, at the headline's step sizes: the production
dispatch (plan height, production epilogues incl. QKV + RoPE), interleaved
rounds in one process, each call on the next of > 1.5 GB of weight copies.

    python tools/bench_gemm_persist.py [out.jsonl] [M,M,...]
"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402
from mcp_amd.ops import reference as ref  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else None
MS = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else \
    [1024, 1536, 2048, 2560, 3072, 3584, 4096]
L = ops.lib()
dev = "cuda"
s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
SHAPES = [("qkv+rope", 6144, 4096), ("o+res", 4096, 4096), ("gate|up", 28672, 4096),
          ("down+res", 4096, 14336)]
Hq, Hkv, D, BS = 32, 8, 128, 64


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
    Ws = [(torch.randn(N, K, device=dev) / math.sqrt(K)).bfloat16()
          for _ in range(max(3, int(1.6e9 // (N * K * 2))))]
    nb = mmax // BS + 2
    kc = torch.zeros(nb, Hkv, BS, D, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    cs = ref.rope_cos_sin(8192, D, 500000.0, dev)
    pos_all = torch.randint(0, 8000, (mmax,), device=dev, dtype=torch.int32)
    slots_all = torch.randperm(nb * BS, device=dev)[:mmax].to(torch.int32)
    for M in MS:
        x = X[:M]
        if L.gemm_select(M, N, K) != 1:
            continue
        if fam == "gate|up":
            y = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
            fn = lambda i: ops.gemm_silu(x, Ws[i], out=y)
        elif fam == "qkv+rope":
            q = torch.empty(M, Hq, D, device=dev, dtype=torch.bfloat16)
            pos, slots = pos_all[:M], slots_all[:M]
            fn = lambda i: ops.qkv_rope(x, Ws[i], pos, slots, cs, q, kc, vc, Hq, Hkv, D)
        else:
            y = R[:M].clone()
            fn = lambda i: ops.gemm(x, Ws[i], R=y, out=y)
        best = {0: float("inf"), 1: float("inf")}
        for _ in range(4):
            for p in (0, 2):
                L.gemm_persist_force(p)
                best[min(p, 1)] = min(best[min(p, 1)], time_us(fn, len(Ws)))
        L.gemm_persist_force(-1)
        f = 2 * M * N * K
        h = {1: 256, 2: 192, 3: 160, 4: 224, 5: 128}.get(L.gemm_plan_lookup(M, N, K), 256)
        tiles = math.ceil(M / h) * (N // 256)
        rec = {"family": fam, "N": N, "K": K, "M": M, "height": h, "tiles": tiles,
               "one_tile_us": round(best[0], 1), "persistent_us": round(best[1], 1),
               "one_tile_tf": round(f / best[0] / 1e6, 1), "persistent_tf": round(f / best[1] / 1e6, 1),
               "speedup": round(best[0] / best[1], 3)}
        print(json.dumps(rec), flush=True)
        if out:
            with open(out, "a") as fh:
                fh.write(json.dumps(rec) + "\n")
    del X, R, Ws, kc, vc
    torch.cuda.empty_cache()
