"""A/B the 256^2 GEMM structural variants in one process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24), random N(0,1) operands."""
import json, sys
import torch
sys.path.insert(0, '.')
import mcp_amd.ops as ops
L = ops.lib()
dev = 'cuda'
shapes = [(4096, 6144, 4096), (4096, 4096, 4096), (4096, 28672, 4096), (4096, 4096, 14336),
          (3584, 6144, 4096), (1792, 6144, 4096)]
variants = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [8, 25, 30, 31, 32, 33]
if len(sys.argv) > 2:                      # "M,N,K;M,N,K;..."
    shapes = [tuple(int(x) for x in sh.split(",")) for sh in sys.argv[2].split(";")]
rounds = 3
res = {}
for (M, N, K) in shapes:
    X = torch.randn(M, K, device=dev).bfloat16()
    W = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
    Y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ref = X.float() @ W.float().t()
    errs = {}
    for v in variants:
        L.gemm_variant(X, W, Y, v)
        errs[v] = ((Y.float() - ref).norm() / ref.norm()).item()
    times = {v: [] for v in variants + ['torch']}
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(rounds):
        for v in variants + ['torch']:
            fn = (lambda: torch.matmul(X, W.t())) if v == 'torch' else (lambda v=v: L.gemm_variant(X, W, Y, v))
            fn(); torch.cuda.synchronize()
            s.record()
            for _ in range(10):
                fn()
            e.record(); torch.cuda.synchronize()
            times[v].append(s.elapsed_time(e) / 10)
    out = {"shape": [M, N, K]}
    for v in variants + ['torch']:
        ms = min(times[v])
        out[str(v)] = round(2 * M * N * K / ms / 1e9, 1)
    out["bad"] = [v for v in variants if errs[v] > 1e-2]
    print(json.dumps(out), flush=True)
