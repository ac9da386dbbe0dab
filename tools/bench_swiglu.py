"""SwiGLU projection (gate|up interleaved, SiLU fused in the epilogue) vs the
plain GEMM of the same shape and torch.matmul, Llama-3-8B gate/up (N = 28672)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402

L = ops.lib()
N, K = 28672, 4096
W = (torch.randn(N, K, device="cuda") / math.sqrt(K)).bfloat16()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def t_us(fn, n=10):
    fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for M in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2048,2600,3000,3500,4096").split(",")]:
    X = torch.randn(M, K, device="cuda").bfloat16()
    Y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    Ys = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
    r = {"M": M}
    for name, fn in [("swiglu", lambda: L.gemm_silu(X, W, Ys)), ("plain", lambda: L.gemm(X, W, Y, None, -1)),
                     ("torch", lambda: torch.matmul(X, W.t()))]:
        us = t_us(fn)
        r[name + "_tf"] = round(2 * M * N * K / us / 1e6, 1)
    print(json.dumps(r), flush=True)
