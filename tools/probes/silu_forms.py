"""Cold-weight decode GEMMs through the skinny kernel at each form
(MCP_SKINNY_FORM, set by the caller): SwiGLU gate|up and the residual down / o."""
import json, os, sys, torch
sys.path.insert(0, os.getcwd())
import mcp_amd.ops as ops
L = ops.lib()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
def t_us(fn, R, n=None):
    n = n or 2 * R
    for i in range(R): fn(i)
    torch.cuda.synchronize(); e0.record()
    for i in range(n): fn(i % R)
    e1.record(); torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / n * 1e3, 1)
form = os.environ.get("MCP_SKINNY_FORM", "default")
for (N, K, silu) in [(28672, 4096, True), (4096, 14336, False), (4096, 4096, False), (6144, 4096, False)]:
    R = int(3.2e9 // (N * K * 2)) + 1
    Ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(R)]
    r = {"form": form, "N": N, "K": K}
    for M in (1, 4, 8, 16):
        X = torch.randn(M, K, device="cuda").bfloat16()
        if silu:
            Y = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
            r[f"M{M}"] = t_us(lambda i: L.gemm_silu(X, Ws[i], Y), R)
        else:
            Y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            r[f"M{M}"] = t_us(lambda i: L.gemm(X, Ws[i], Y, None, 2), R)
    print(json.dumps(r), flush=True)
    del Ws
