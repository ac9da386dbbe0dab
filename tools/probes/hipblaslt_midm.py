"""hipBLASLt's own kernels for the gate|up GEMM at mid M (the yardstick of
VERDICT r5 next #3): run torch.matmul at M = 192 / 256 / 320 under
``rocprofv3 --kernel-trace --stats`` and read the chosen kernels' names (macro
tile, split) and times from the trace.  Synthetic data, cold weights."""
import torch

N, K = 28672, 4096
Ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16().t() for _ in range(6)]
for M in (192, 256, 320):
    X = torch.randn(M, K, device="cuda").bfloat16()
    P = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for i in range(24):
        torch.matmul(X, Ws[i % 6], out=P)
    torch.cuda.synchronize()
    print(M, "done", flush=True)
