"""GEMM microbenchmark: our 128^2 and 256^2 MFMA kernels vs torch.matmul
(hipBLASLt) on the Llama-3-8B projection shapes.  Random N(0,1) operands
(cdna_hip_programming.md §5.4 rule 25: never zero-filled)."""
import json, sys, time
import torch
sys.path.insert(0, '.')
import mcp_amd.ops as ops

dev = 'cuda'
shapes = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]
Ms = [int(x) for x in (sys.argv[1].split(',') if len(sys.argv) > 1 else ['1024', '2048', '4096', '8192'])]
res = []

def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters

for M in Ms:
    for N, K in shapes:
        X = torch.randn(M, K, device=dev).bfloat16()
        W = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
        Y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ref = (X.float() @ W.float().t())
        row = {"M": M, "N": N, "K": K}
        for algo in (0, 1):
            ops.gemm(X, W, out=Y, algo=algo)
            err = ((Y.float() - ref).norm() / ref.norm()).item()
            ms = timeit(lambda: ops.gemm(X, W, out=Y, algo=algo))
            row[f"a{algo}_tf"] = round(2 * M * N * K / ms / 1e9, 1)
            row[f"a{algo}_err"] = round(err, 5)
        ms = timeit(lambda: torch.matmul(X, W.t()))
        row["torch_tf"] = round(2 * M * N * K / ms / 1e9, 1)
        row["auto"] = ops.lib().gemm_select(M, N, K)
        res.append(row)
        print(json.dumps(row), flush=True)
