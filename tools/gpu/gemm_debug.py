import sys, torch
sys.path.insert(0, '.')
import mcp_amd.ops as ops
L = ops.lib()
torch.manual_seed(0)
for (M, N, K) in [(256, 256, 128), (256, 256, 256), (512, 512, 1024)]:
    X = torch.randn(M, K, device='cuda').bfloat16()
    W = torch.randn(N, K, device='cuda').bfloat16()
    ref = X.float() @ W.float().t()
    for v in (49, 51):
        Y = torch.zeros(M, N, device='cuda', dtype=torch.bfloat16)
        L.gemm_variant(X, W, Y, v)
        torch.cuda.synchronize()
        err = (Y.float() - ref).abs()
        bad = (err > 0.05 * ref.abs().max()).float()
        rows = bad.sum(1).nonzero().flatten().tolist()
        cols = bad.sum(0).nonzero().flatten().tolist()
        print(M, N, K, v, "relerr", float((Y.float()-ref).norm()/ref.norm()), "bad rows", rows[:8], len(rows), "bad cols", cols[:8], len(cols), flush=True)
        # try: is it a k-step mixup? compare against partial sums
