"""Measure, per 64-row M bucket, whether hipBLASLt's GEMM with its beta = 1
epilogue (``x.addmm_(a, W.t())``) beats our planned MFMA path with the fused
residual epilogue on the residual projections (o: 4096 x 4096, down:
4096 x 14336), and record the answer as ``"lib"`` in the GEMM plan
(ops/gemm_plan_gfx950.json; ops.gemm routes those buckets to the library).
For the QKV projection (6144 x 4096) the comparison is our whole
``qkv_rope`` (RoPE + paged K/V write fused in the AGPR epilogue, or GEMM +
``rope_kv`` on the other paths) against hipBLASLt's GEMM + our ``rope_kv``.
Cold weights (each call reads the next of > 1.2 GB of weight copies); the
library wins a bucket only when it is > 3 % faster (hysteresis against noise).

    python tools/tune_gemm_lib.py [plan.json] [m_max]
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402
from mcp_amd.ops import reference as ref  # noqa: E402

ops._LIB_ON = False                       # time our kernels, not an old "lib" plan
path = sys.argv[1] if len(sys.argv) > 1 else ops.GEMM_PLAN_FILE
m_max = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
only = {tuple(int(v) for v in x.split("x")) for x in sys.argv[3].split(",")} if len(sys.argv) > 3 else None
plan = json.load(open(path))
ops.lib()
dev = "cuda"
s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def time_us(fn, n, reps=6):
    fn(0)
    best = float("inf")
    for _ in range(3):
        s_ev.record()
        for i in range(reps):
            fn(i % n)
        e_ev.record()
        torch.cuda.synchronize()
        best = min(best, s_ev.elapsed_time(e_ev) * 1e3 / reps)
    return best


t0 = time.time()
for sh in plan["shapes"]:
    N, K = sh["N"], sh["K"]
    if (N, K) not in ((4096, 4096), (4096, 14336), (6144, 4096),
                      (8192, 8192), (8192, 28672), (10240, 8192)):
        continue
    if only is not None and (N, K) not in only:
        continue
    qkv_shape = (N, K) in ((6144, 4096), (10240, 8192))
    Hq = N // 128 - 16                     # 8 kv heads of d = 128 (Llama-3 8B / 70B)
    X = torch.randn(m_max, K, device=dev).bfloat16()
    Y = torch.randn(m_max, N, device=dev).bfloat16()
    Ws = [(torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
          for _ in range(max(2, int(1.2e9 // (N * K * 2))))]
    if qkv_shape:                          # Hq q / 8 kv heads, d = 128, 64-token blocks
        nb = m_max // 64 + 1
        rope = (torch.empty(m_max, Hq, 128, device=dev, dtype=torch.bfloat16),
                torch.zeros(nb, 8, 64, 128, device=dev, dtype=torch.bfloat16),
                torch.zeros(nb, 8, 64, 128, device=dev, dtype=torch.bfloat16),
                torch.arange(m_max, device=dev, dtype=torch.int32) % 8000,
                torch.arange(m_max, device=dev, dtype=torch.int32))
        Q = torch.empty(m_max, N, device=dev, dtype=torch.bfloat16)
        cs = ref.rope_cos_sin(8192, 128, 500000.0, dev)
    lib, us = [], []
    for b in range(m_max // 64):
        M = (b + 1) * 64
        x, y = X[:M], Y[:M]
        if qkv_shape:
            q, kc, vc, pos, slots, qkv = rope[0][:M], rope[1], rope[2], rope[3][:M], rope[4][:M], Q[:M]
            ours = time_us(lambda i: ops.qkv_rope(x, Ws[i], pos, slots, cs, q, kc, vc, Hq, 8, 128,
                                                  qkv=qkv), len(Ws))
            blas = time_us(lambda i: (torch.matmul(x, Ws[i].t(), out=qkv),
                                      ops.rope_kv(qkv, pos, slots, cs, q, kc, vc, Hq, 8, 128)), len(Ws))
        else:
            ours = time_us(lambda i: ops.gemm(x, Ws[i], R=y, out=y), len(Ws))
            blas = time_us(lambda i: y.addmm_(x, Ws[i].t()), len(Ws))
        lib.append(1 if blas < 0.97 * ours else 0)
        us.append([round(ours, 1), round(blas, 1)])
    sh["lib"] = lib
    sh["lib_us"] = us
    print(json.dumps({"N": N, "K": K, "lib": lib, "s": round(time.time() - t0, 1)}), flush=True)
    del X, Y, Ws
plan["lib"] = ("1 = hipBLASLt addmm_ (beta = 1) for this residual bucket, measured > 3 % faster "
               "(tools/tune_gemm_lib.py; lib_us = [ours, hipBLASLt] us, cold weights)")
with open(path, "w") as f:
    json.dump(plan, f, indent=None, separators=(",", ":"))
    f.write("\n")
print(json.dumps({"written": path, "s": round(time.time() - t0, 1)}), flush=True)
