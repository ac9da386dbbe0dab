"""M = 193-255 (bucket 3): gemm_select sends these to the 128^2 path whatever
the plan's code for the bucket (timed at M = 256, where the AGPR height is
used).  Cold-weight times of production vs the AGPR heights at these M."""
import json, os, sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import mcp_amd.ops as ops
L = ops.lib()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
def t_us(fn, R, n=24):
    for i in range(R): fn(i)
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(3):
        e0.record()
        for i in range(n): fn(i % R)
        e1.record(); torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / n * 1e3)
    return round(best, 1)
for name, N, K, kind in (("gate_up", 28672, 4096, "silu"), ("o", 4096, 4096, "res"), ("down", 4096, 14336, "res"), ("qkv", 6144, 4096, "plain")):
    R = max(2, int(1.5e9 // (N * K * 2)))
    Ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(R)]
    for M in (193, 208, 224, 240, 255, 256):
        X = torch.randn(M, K, device="cuda").bfloat16()
        ss = (X.float().pow(2).sum(-1) * (1 << 20)).to(torch.int64)
        out = {"shape": name, "M": M}
        if kind == "silu":
            Y = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
            out["prod"] = t_us(lambda i: L.gemm_silu(X, Ws[i], Y, ss, 1e-5), R)
            for c in (1, 2, 3, 4, 5):
                if L.gemm_silu_algo(X, Ws[0], Y, c, ss, 1e-5) == 0:
                    out[f"agpr{c}"] = t_us(lambda i, c=c: L.gemm_silu_algo(X, Ws[i], Y, c, ss, 1e-5), R)
        else:
            Y = torch.randn(M, N, device="cuda").bfloat16()
            Rr = Y if kind == "res" else None
            so = torch.zeros(M, dtype=torch.int64, device="cuda") if kind == "res" else None
            out["prod"] = t_us(lambda i: L.gemm(X, Ws[i], Y, Rr, -1, so), R)
            for c in (1, 2, 3, 4, 5):
                out[f"agpr{c}"] = t_us(lambda i, c=c: L.gemm(X, Ws[i], Y, Rr, 8 + c, so), R)
        print(json.dumps(out), flush=True)
    del Ws
