"""Fused vs GEMM + segmented top-k latency across corpus sizes (MI355X), to
place the retrieval index's path switch.  python tools/topk_size_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402

dev = "cuda"
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def t_ms(fn, n=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / n, 4)


for N in (1000, 10000, 50000, 100000, 300000, 1000000):
    corpus = torch.randn(N, 1024, device=dev).bfloat16()
    ops.l2norm_rows(corpus)
    for B in (1, 16, 64):
        q = torch.randn(B, 1024, device=dev).bfloat16()
        ops.l2norm_rows(q)
        vf, _ = ops.topk_cosine(q, corpus, 32, fused=True)
        vg, _ = ops.topk_cosine(q, corpus, 32, fused=False)
        print(json.dumps({"N": N, "B": B, "fused_ms": t_ms(lambda: ops.topk_cosine(q, corpus, 32, fused=True)),
                          "gemm_ms": t_ms(lambda: ops.topk_cosine(q, corpus, 32, fused=False)),
                          "agree": bool(torch.allclose(vf, vg, atol=1e-4))}), flush=True)
