"""Run one GEMM variant a few times (for rocprofv3 --pmc passes)."""
import sys, torch
sys.path.insert(0, '.')
import mcp_amd.ops as ops
v, M, N, K = (int(x) for x in sys.argv[1:5])
L = ops.lib()
X = torch.randn(M, K, device='cuda').bfloat16()
W = (torch.randn(N, K, device='cuda') / K ** 0.5).bfloat16()
Y = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
for _ in range(6):
    if v < 0:
        torch.matmul(X, W.t())
    else:
        L.gemm_variant(X, W, Y, v)
torch.cuda.synchronize()
