"""gate|up (SwiGLU epilogue) at mid M, cold weights, through the production
dispatch; run once per setting of the static GEMM knobs (MCP_GEMM_HYBRID,
MCP_GEMM_TAIL_SPLIT) to compare the tail handling of partial waves.

    MCP_GEMM_HYBRID=0 python tools/bench_swiglu_mid.py [m0 m1 step]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402

m0, m1, mstep = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (1600, 4096, 64)
N, K = 28672, 4096
X = torch.randn(m1, K, device="cuda").bfloat16()
Ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(6)]
Y = torch.empty(m1, N // 2, device="cuda", dtype=torch.bfloat16)
s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
tag = {k: os.environ.get(k) for k in ("MCP_GEMM_HYBRID", "MCP_GEMM_TAIL_SPLIT", "MCP_GEMM_BM")}
for M in range(m0, m1 + 1, mstep):
    x, y = X[:M], Y[:M]
    best = float("inf")
    ops.gemm_silu(x, Ws[0], out=y)
    for _ in range(3):
        s_ev.record()
        for i in range(6):
            ops.gemm_silu(x, Ws[i], out=y)
        e_ev.record()
        torch.cuda.synchronize()
        best = min(best, s_ev.elapsed_time(e_ev) * 1e3 / 6)
    print(json.dumps({**tag, "M": M, "us": round(best, 1), "tf": round(2 * M * N * K / best / 1e6, 1)}),
          flush=True)
