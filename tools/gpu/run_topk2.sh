set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench_suite.py topk --n 10000000 > gpurun_out/topk_10m.jsonl 2>&1; cat gpurun_out/topk_10m.jsonl
timeout -k 10 300 python -u - > gpurun_out/topk_probe.txt 2>&1 <<'PY'
import torch, mcp_amd.ops as ops
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
n, dim, k, b = 10_000_000, 1024, 32, 64
corpus = torch.randn(n, dim, device=dev, generator=g).bfloat16(); ops.l2norm_rows(corpus)
for bb in (1, 16):
    torch.randn(bb, dim, device=dev, generator=g)
q = torch.randn(b, dim, device=dev, generator=g).bfloat16(); ops.l2norm_rows(q)
v, i = ops.topk_cosine(q, corpus, k)
vu, iu = ops.topk_cosine(q, corpus, k, fused=False)
direct = (q.float().unsqueeze(1) * corpus[i.long()].float()).sum(-1)
print("fused vs direct", float((direct - v).abs().max()))
print("fused vs unfused values", float((v - vu).abs().max()))
big = q.float() @ corpus.float().t()
print("torch big-gemm scores at fused idx vs direct", float((big.gather(1, i.long()) - direct).abs().max()))
PY
cat gpurun_out/topk_probe.txt
