"""Cold-weight probe: flex tiles with S-way split-K (fp32 partials + the
reduce; algo 1000 + 16 cand + S) against the shipped dispatch for the narrow
projections at serving M (config 5 runs M = 129-384 most of the time,
profiles/config5_gemm_mhist_r4.md).  Checks the winner against fp32.
    python tools/bench_flex_split_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402
from mcp_amd.ops import reference as ref  # noqa: E402

L = ops.lib()
L.gemm_splitk_init(256 << 20)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
TILES = [(64, 64), (64, 128), (64, 160), (96, 64), (96, 128), (128, 96), (128, 128), (128, 160),
         (128, 192), (256, 32), (192, 128), (160, 128), (256, 64), (192, 64)]


def t_us(fn, R, n=20):
    for i in range(R):
        fn(i)
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(2):
        e0.record()
        for i in range(n):
            fn(i % R)
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / n * 1e3)
    return round(best, 1)


MS = [int(m) for m in os.environ.get("PROBE_MS", "128,192,256,320,384").split(",")]
SHAPES = [(4096, 14336, True), (4096, 4096, True), (6144, 4096, False)]
if os.environ.get("PROBE_WIDE") == "1":
    SHAPES.append((28672, 4096, False))
for (N, K, res) in SHAPES:
    R = max(4, int(1.6e9 // (N * K * 2)) + 1)
    Ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(R)]
    for M in MS:
        X = torch.randn(M, K, device="cuda").bfloat16()
        Y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        Rr = torch.randn(M, N, device="cuda").bfloat16() if res else None
        r = {"M": M, "N": N, "K": K, "floor_us": round(N * K * 2 / 6.0e12 * 1e6, 1),
             "auto_us": t_us(lambda i: L.gemm(X, Ws[i], Y, Rr, -1), R)}
        if N == 28672:                     # gate|up: the shipped SwiGLU dispatch
            Yh = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
            r["auto_silu_us"] = t_us(lambda i: L.gemm_silu(X, Ws[i], Yh, None, 0.0), R)
        best = None
        for c, (tm, tn) in enumerate(TILES):
            tiles = -(-M // tm) * -(-N // tn)
            for S in (2, 3, 4, 7, 8):
                if (K // 64) % S or not (64 <= tiles * S <= 1024):
                    continue
                t = t_us(lambda i: L.gemm(X, Ws[i], Y, Rr, 1000 + 16 * c + S), R)
                if best is None or t < best[0]:
                    best = (t, c, S)
        if best:
            r["best_split_us"], r["cand"], r["S"] = best
            r["tile"] = TILES[best[1]]
            Yc = torch.empty_like(Y)
            Rc = Rr.clone() if res else None
            L.gemm(X, Ws[0], Yc, Rc, 1000 + 16 * best[1] + best[2])
            e = ref.gemm(X, Ws[0], Rr)
            r["rel_err"] = round(((Yc.float() - e).norm() / e.norm()).item(), 5)
        print(json.dumps(r), flush=True)
    del Ws
