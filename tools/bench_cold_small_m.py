"""Small-M projections with COLD weights (serving reality: the 16 GB model
streams through HBM every step, nothing stays in the 256 MB Infinity Cache):
each call uses the next of R distinct weight copies (> 1.5 GB in total).
Times every path a decode-sized step can take.
    python tools/bench_cold_small_m.py [M,M,...]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402

L = ops.lib()
Ms = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 4, 8, 16, 32, 48, 64, 96, 128]
SHAPES = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]
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


for (N, K) in SHAPES:
    R = max(4, int(1.6e9 // (N * K * 2)) + 1)
    Ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(R)]
    for M in Ms:
        X = torch.randn(M, K, device="cuda").bfloat16()
        Y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        r = {"M": M, "N": N, "K": K, "copies": R}
        for name, algo in (("auto", -1), ("128", 0), ("stream", 3), ("skinny", 2)):
            if algo == 2 and M > 128:
                continue
            try:
                r[name + "_us"] = t_us(lambda i, a=algo: L.gemm(X, Ws[i], Y, None, a), R)
            except Exception as e:  # noqa: BLE001
                r[name + "_us"] = None
        if N == 28672:
            Ys = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
            r["swiglu_auto_us"] = t_us(lambda i: L.gemm_silu(X, Ws[i], Ys), R)
        r["torch_us"] = t_us(lambda i: torch.matmul(X, Ws[i].t()), R)
        r["floor_us"] = round(N * K * 2 / 6.0e12 * 1e6, 1)
        print(json.dumps(r), flush=True)
    del Ws
