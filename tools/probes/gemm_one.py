import sys, torch
sys.path.insert(0, '.')
import mcp_amd.ops as ops
M, N, K, v = [int(x) for x in sys.argv[1:5]]
X = torch.randn(M, K, device='cuda').bfloat16()
W = (torch.randn(N, K, device='cuda') / K ** 0.5).bfloat16()
Y = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
for _ in range(int(sys.argv[5]) if len(sys.argv) > 5 else 5):
    if v < 0:
        torch.matmul(X, W.t())
    else:
        ops.lib().gemm_variant(X, W, Y, v)
torch.cuda.synchronize()
