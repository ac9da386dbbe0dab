"""Small-M projection GEMMs (decode / tail steps of the headline bench): time
the kernels each entry point can pick at the Llama-3-8B weight shapes.
    MCP_GEMM_SPLITK128=0|1 python tools/bench_small_m.py [M,M,...]
algo 0 = 128^2 kernel (split-K when enabled and the tiles do not fill the
chip), 1 = 256 path, 2 = skinny (M <= 128), -1 = production selection; plus
the SwiGLU entry point (gate|up interleaved) and torch.matmul (hipBLASLt)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402

L = ops.lib()
Ms = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [32, 64, 128, 192, 256, 320, 512, 768, 1024]
SHAPES = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def t_us(fn, n=20):
    fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / n * 1e3, 1)


for (N, K) in SHAPES:
    W = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    for M in Ms:
        X = torch.randn(M, K, device="cuda").bfloat16()
        Y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ref = X.float() @ W.float().t()
        r = {"M": M, "N": N, "K": K, "splitk128": os.environ.get("MCP_GEMM_SPLITK128", "1"),
             "splits": L.gemm128_splits(M, N, K)}
        for algo in ([0, 1, -1] + ([2] if M <= 128 else [])):
            if algo == 1 and (K % 128 or N % 256) and M < 256:
                pass
            L.gemm(X, W, Y, None, algo)
            err = ((Y.float() - ref).norm() / ref.norm()).item()
            r[f"a{algo}_us"] = t_us(lambda: L.gemm(X, W, Y, None, algo))
            r[f"a{algo}_err"] = round(err, 5)
        if N == 28672:
            Ys = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
            r["swiglu_us"] = t_us(lambda: L.gemm_silu(X, W, Ys))
        r["torch_us"] = t_us(lambda: torch.matmul(X, W.t()))
        r["GBps_weights_auto"] = round(N * K * 2 / r["a-1_us"] / 1e3, 0)
        print(json.dumps(r), flush=True)
