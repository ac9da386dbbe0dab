"""The headline's four projection families at M = 2560 through the production
dispatch (plan heights, production epilogues), 6 launches each, for a
rocprofv3 --pmc pass (tools/gpu_run.sh pmc, tools/pmc_summary.py)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402
from mcp_amd.ops import reference as ref  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 2560
dev = "cuda"
Hq, Hkv, D, BS = 32, 8, 128, 64
for fam, N, K in (("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)):
    x = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) / math.sqrt(K)).bfloat16()
    if fam == "gate_up":
        fn = lambda: ops.gemm_silu(x, w)
    elif fam == "qkv":
        nb = M // BS + 2
        kc = torch.zeros(nb, Hkv, BS, D, device=dev, dtype=torch.bfloat16)
        vc = torch.zeros_like(kc)
        q = torch.empty(M, Hq, D, device=dev, dtype=torch.bfloat16)
        cs = ref.rope_cos_sin(8192, D, 500000.0, dev)
        pos = torch.randint(0, 8000, (M,), device=dev, dtype=torch.int32)
        slots = torch.randperm(nb * BS, device=dev)[:M].to(torch.int32)
        fn = lambda: ops.qkv_rope(x, w, pos, slots, cs, q, kc, vc, Hq, Hkv, D)
    else:
        y = torch.randn(M, N, device=dev).bfloat16()
        fn = lambda: ops.gemm(x, w, R=y, out=y)
    for _ in range(6):
        fn()
    torch.cuda.synchronize()
print("pmc gemm head done")
