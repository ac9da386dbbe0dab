"""Which hipBLASLt kernels torch.matmul picks at the serving-size M (names via rocprofv3)."""
import torch
for M in (256, 384, 512, 768, 1024):
    X = torch.randn(M, 4096, device='cuda').bfloat16()
    for N in (6144, 4096):
        W = torch.randn(N, 4096, device='cuda').bfloat16()
        for _ in range(3):
            torch.matmul(X, W.t())
        torch.cuda.synchronize()
