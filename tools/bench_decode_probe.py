"""Cold-weight timing of the decode-sized projections at the M a single
intent's steps run (1 decision + its forced span: 5-17 tokens): the dispatch
as shipped, and the weight-streaming kernel at forced split counts.
MCP_PROBE_SKINNY_X1=1 (timing probe, wrong results) makes every token row of
the skinny kernel load X row 0, to price the activation loads.
    python tools/bench_decode_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402

L = ops.lib()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
TAG = os.environ.get("PROBE_TAG", "")


def t_us(fn, R, n=28):
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


for (N, K, kind) in [(28672, 4096, "swiglu"), (4096, 14336, "res"), (6144, 4096, "plain"),
                     (4096, 4096, "res")]:
    R = max(4, int(1.6e9 // (N * K * 2)) + 1)
    Ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(R)]
    for M in (1, 4, 8, 12, 16):
        X = torch.randn(M, K, device="cuda").bfloat16()
        Y = torch.empty(M, N // 2 if kind == "swiglu" else N, device="cuda", dtype=torch.bfloat16)
        Rr = torch.randn(M, N, device="cuda").bfloat16() if kind == "res" else None
        r = {"tag": TAG, "M": M, "N": N, "K": K, "kind": kind, "floor_us": round(N * K * 2 / 6.0e12 * 1e6, 1)}
        if kind == "swiglu":
            r["auto_us"] = t_us(lambda i: L.gemm_silu(X, Ws[i], Y, None, 0.0), R)
            if M > 8:                      # the stream kernel serves 9..32 (gemm_stream_pick)
                for S in (1, 2, 3, 4, 6):
                    L.gemm_stream_force_splits(S)
                    r[f"stream_s{S}_us"] = t_us(lambda i: L.gemm_silu(X, Ws[i], Y, None, 0.0), R)
                L.gemm_stream_force_splits(0)
        else:
            r["auto_us"] = t_us(lambda i: L.gemm(X, Ws[i], Y, Rr, -1), R)
            r["skinny_us"] = t_us(lambda i: L.gemm(X, Ws[i], Y, Rr, 2), R)
            for S in (1, 2, 4, 8):
                L.gemm_stream_force_splits(S)
                r[f"stream_s{S}_us"] = t_us(lambda i: L.gemm(X, Ws[i], Y, Rr, 3), R)
            L.gemm_stream_force_splits(0)
        print(json.dumps(r), flush=True)
    del Ws
