import torch
X = torch.randn(4096, 4096, device='cuda').bfloat16()
for N in (28672, 6144, 4096):
    W = torch.randn(N, 4096, device='cuda').bfloat16()
    for _ in range(3):
        torch.matmul(X, W.t())
torch.cuda.synchronize()
