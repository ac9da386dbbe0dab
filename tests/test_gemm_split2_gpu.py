"""K-half split form of the AGPR GEMM (csrc/gemm256d.hip SPLIT 2: two
workgroups per tile, the in-launch sc1 hand-off, the slab added in the wide
epilogue) against the plain-PyTorch fp32 reference: every tile height, plain /
+ residual / SwiGLU with the fused-norm scale, back-to-back launches (the
tile counters re-arm themselves) and hipGraph replays.  MI355X only."""
import math

import pytest
import torch

import mcp_amd.ops as ops
from mcp_amd.ops import reference as ref

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")]

DEV = "cuda"
HEIGHTS = (256, 224, 192, 160, 128)


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.fixture(params=[0, 1], ids=["pf0", "pf1"])
def w_prefetch(request):
    """The split form with and without the W L2 fills ahead of the DMA (PF)."""
    L = ops.lib()
    L.gemm_pf_force(request.param)
    yield request.param
    L.gemm_pf_force(-1)


@pytest.mark.parametrize("M,N,K", [(256, 3584, 4096), (200, 2048, 1024), (97, 4096, 14336),
                                   (300, 1024, 512)])
def test_split2_plain_and_residual(M, N, K, w_prefetch):
    torch.manual_seed(11)
    L = ops.lib()
    X = torch.randn(M, K, device=DEV).bfloat16()
    W = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    R = torch.randn(M, N, device=DEV).bfloat16()
    exp = X.float() @ W.float().t()
    ran = 0
    for bm in HEIGHTS:
        Y = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
        if L.gemm_split2(X, W, Y, None, bm):
            continue                                   # more tiles than one wave holds
        torch.cuda.synchronize()
        assert rel_err(Y, exp) < 1e-2, bm
        Y2 = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
        assert L.gemm_split2(X, W, Y2, R, bm) == 0
        torch.cuda.synchronize()
        assert rel_err(Y2, exp + R.float()) < 1e-2, bm
        ran += 1
    assert ran >= 3


@pytest.mark.parametrize("M", [129, 192, 256, 320])
def test_split2_swiglu_every_height(M, w_prefetch):
    """gate|up + SwiGLU with the fused-norm row scale (the 'silu' plan codes
    401-405), N = 28672 as in Llama-3-8B where the tiles fit one wave."""
    torch.manual_seed(12)
    L = ops.lib()
    F, K = 14336, 4096
    X = torch.randn(M, K, device=DEV).bfloat16()
    g = (torch.randn(F, K, device=DEV) / math.sqrt(K)).bfloat16()
    u = (torch.randn(F, K, device=DEV) / math.sqrt(K)).bfloat16()
    W = ref.interleave_gate_up(g, u).contiguous()
    eps = 1e-5
    ss = (X.float().pow(2).sum(-1) * (1 << 20)).round().to(torch.int64)
    rs = torch.rsqrt(ss.double() / (1 << 20) / K + eps).float()[:, None]
    exp = torch.nn.functional.silu((X.float() @ g.float().t()) * rs) * ((X.float() @ u.float().t()) * rs)
    ran = 0
    for code in range(400, 406):
        Y = torch.full((M, F), float("nan"), device=DEV, dtype=torch.bfloat16)
        if L.gemm_silu_algo(X, W, Y, code, ss, eps):
            continue
        torch.cuda.synchronize()
        assert rel_err(Y, exp) < 2e-2, code
        ran += 1
    assert ran >= (1 if M <= 256 else 0)            # past 256 rows the tiles exceed one wave


def test_split2_back_to_back_and_graph(w_prefetch):
    """Many launches in a row and inside a hipGraph: every tile's last arriver
    re-arms its counter, so each launch sees fresh tickets (a stale counter
    would make a first arriver wait for a partner slab that never comes, and
    return wrong sums after the bounded poll)."""
    torch.manual_seed(13)
    L = ops.lib()
    M, N, K = 256, 3584, 2048
    X = torch.randn(M, K, device=DEV).bfloat16()
    Ws = [(torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16() for _ in range(3)]
    exps = [X.float() @ w.float().t() for w in Ws]
    Ys = [torch.empty(M, N, device=DEV, dtype=torch.bfloat16) for _ in Ws]
    for rep in range(20):
        for w, y in zip(Ws, Ys):
            assert L.gemm_split2(X, w, y, None, 256 if rep % 2 else 128) == 0
    torch.cuda.synchronize()
    for y, e in zip(Ys, exps):
        assert rel_err(y, e) < 1e-2
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        for y in Ys:
            y.zero_()
        with torch.cuda.graph(graph, stream=s):
            for w, y in zip(Ws, Ys):
                L.gemm_split2(X, w, y, None, 192)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(5):
        for y in Ys:
            y.fill_(float("nan"))
        graph.replay()
        torch.cuda.synchronize()
        for y, e in zip(Ys, exps):
            assert rel_err(y, e) < 1e-2
