"""QKV projection + RoPE + paged K/V write: fused epilogue vs GEMM + rope_kv.
    python tools/bench_qkv_rope.py [M,M,...]"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402
from mcp_amd.ops import reference as ref  # noqa: E402

L = ops.lib()
Hq, Hkv, D, H, BS = 32, 8, 128, 4096, 64
W = (torch.randn((Hq + 2 * Hkv) * D, H, device="cuda") / math.sqrt(H)).bfloat16()
cs = ref.rope_cos_sin(8192, D, 500000.0, "cuda")
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


for M in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1536,2048,2600,3072,4096").split(",")]:
    X = torch.randn(M, H, device="cuda").bfloat16()
    nb = (M + BS - 1) // BS
    pos = torch.arange(M, device="cuda", dtype=torch.int32) % 8000
    slots = torch.arange(M, device="cuda", dtype=torch.int32)
    q = torch.empty(M, Hq, D, device="cuda", dtype=torch.bfloat16)
    kc = torch.empty(nb, Hkv, BS, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.empty_like(kc)
    qkv = torch.empty(M, W.shape[0], device="cuda", dtype=torch.bfloat16)
    fused = t_us(lambda: L.qkv_rope(X, W, qkv, pos, slots, cs, q, kc, vc, Hq, Hkv, D))
    sep = t_us(lambda: (L.gemm(X, W, qkv, None, -1),
                        L.rope_kv(qkv, pos, slots, cs, q, kc, vc, Hq, Hkv, D)))
    gemm = t_us(lambda: L.gemm(X, W, qkv, None, -1))
    print(json.dumps({"M": M, "fused_us": fused, "gemm_plus_rope_us": sep, "gemm_only_us": gemm,
                      "selected_256": L.gemm_select(M, W.shape[0], H)}), flush=True)
