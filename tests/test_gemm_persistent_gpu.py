"""Persistent AGPR GEMM (csrc/gemm256p.hip) against fp32, every epilogue at
every tile height: plain, residual in place with the fused
RMSNorm statistic (ss_out), SwiGLU with the fused norm scale (ss_in), and
QKV + RoPE + paged K/V write.  Shapes give several tiles per workgroup (the
next tile's operands prefetched by the previous one, stores drained under the
next mainloop), a last M tile that is partial (range-checked stores), and a
grid smaller than the CU count.  Repeated runs are bitwise equal, and the
residual statistic equals the one-tile kernel's bit for bit (tile heights
below 256 rows, whose one-tile dispatch has no stream-K form)."""
import math

import pytest
import torch

import mcp_amd.ops as ops
from mcp_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
CODES = (1, 2, 3, 4, 5)          # 256 / 192 / 160 / 224 / 128-row tiles


def rel_err(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-6)).item()


@pytest.fixture
def persist():
    L = ops.lib()
    L.gemm_persist_force(2)
    try:
        yield L
    finally:
        L.gemm_persist_force(-1)
        L.gemm_plan_clear()
        ops._load_gemm_plan(L)


@pytest.mark.parametrize("M,N,K", [(1000, 4096, 1024), (2600, 6144, 512), (300, 2048, 4096)])
def test_persistent_plain_and_residual(M, N, K, persist):
    L = persist
    torch.manual_seed(41)
    X = torch.randn(M, K, device=DEV).bfloat16()
    W = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    R = torch.randn(M, N, device=DEV).bfloat16()
    exp = ref.gemm(X, W)
    exp_r = ref.gemm(X, W, R)
    for code in CODES:
        L.gemm_plan_set(N, K, [code] * 128)
        outs = [ops.gemm(X, W) for _ in range(2)]
        assert rel_err(outs[0], exp) < 1e-2, code
        assert torch.equal(outs[0], outs[1]), code
        y = R.clone()
        ss = torch.zeros(M, dtype=torch.int64, device=DEV)
        ops.gemm(X, W, R=y, out=y, ss_out=ss)
        assert rel_err(y, exp_r) < 1e-2, code
        e_ss = y.double().pow(2).sum(-1) * ref.SS_FIX
        assert ((ss.double() - e_ss).abs() / e_ss).max().item() < 1e-5, code
        # the same result and statistic as the one-tile kernel, bit for bit
        # (256-row tiles excepted: that dispatch sends small grids and tail
        # waves through the stream-K kernel, another summation order)
        L.gemm_persist_force(0)
        y1 = R.clone()
        ss1 = torch.zeros(M, dtype=torch.int64, device=DEV)
        ops.gemm(X, W, R=y1, out=y1, ss_out=ss1)
        L.gemm_persist_force(2)
        if code != 1:
            assert torch.equal(y, y1) and torch.equal(ss, ss1), code


@pytest.mark.parametrize("M", [700, 2600])
def test_persistent_swiglu_fused_norm(M, persist):
    L = persist
    torch.manual_seed(42)
    H, F, eps = 1024, 3584, 1e-5
    x = (torch.randn(M, H, device=DEV) * 3).bfloat16()
    gw = torch.rand(H, device=DEV) + 0.5
    ss = ref.row_sumsq(x.cpu()).to(DEV)
    xn = x.float() * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + eps) * gw
    Wg = (torch.randn(2 * F, H, device=DEV) / math.sqrt(H)).bfloat16()
    Wf = (Wg.float() * gw).bfloat16()
    g, u = ref.deinterleave_gate_up(Wg.float())
    e = torch.nn.functional.silu(xn @ g.t()) * (xn @ u.t())
    e_plain = torch.nn.functional.silu(x.float() @ g.t()) * (x.float() @ u.t())
    for code in CODES:
        L.gemm_plan_set(2 * F, H, [code] * 128)
        ys = [ops.gemm_silu(x, Wf, ss_in=ss, eps=eps) for _ in range(2)]
        assert rel_err(ys[0], e) < 2e-2, code
        assert torch.equal(ys[0], ys[1]), code
        assert rel_err(ops.gemm_silu(x, Wg), e_plain) < 2e-2, code


@pytest.mark.parametrize("M", [1024, 2600])
def test_persistent_qkv_rope(M, persist):
    L = persist
    torch.manual_seed(43)
    Hq, Hkv, D, H, BS = 32, 8, 128, 1024, 64
    N = (Hq + 2 * Hkv) * D
    X = torch.randn(M, H, device=DEV).bfloat16()
    W = (torch.randn(N, H, device=DEV) / math.sqrt(H)).bfloat16()
    nb = (M + BS - 1) // BS + 1
    pos = torch.randint(0, 8000, (M,), device=DEV, dtype=torch.int32)
    slots = torch.randperm(nb * BS, device=DEV)[:M].to(torch.int32)
    slots[::7] = -1                                  # rows whose K / V are not written
    cs = ref.rope_cos_sin(8192, D, 500000.0, DEV)
    qkv = ref.gemm(X, W).cpu()
    qr, kr, vr = (torch.zeros(M, Hq, D), torch.zeros(nb, Hkv, BS, D), torch.zeros(nb, Hkv, BS, D))
    ref.rope_kv(qkv, pos.cpu(), slots.cpu(), cs.cpu(), qr, kr, vr, Hq, Hkv, D)
    for code in CODES:
        L.gemm_plan_set(N, H, [code] * 128)
        q = torch.empty(M, Hq, D, device=DEV, dtype=torch.bfloat16)
        kc = torch.zeros(nb, Hkv, BS, D, device=DEV, dtype=torch.bfloat16)
        vc = torch.zeros_like(kc)
        ops.qkv_rope(X, W, pos, slots, cs, q, kc, vc, Hq, Hkv, D)
        assert rel_err(q.cpu(), qr) < 1e-2, code
        assert rel_err(kc.cpu(), kr) < 1e-2 and rel_err(vc.cpu(), vr) < 1e-2, code


def test_persistent_dispatch_rule(persist):
    """Mode 1 (the plan / MCP_GEMM_PERSIST=1 rule) takes the persistent form
    only when the tiles exceed one wave of workgroups."""
    L = persist
    L.gemm_persist_force(1)
    assert L.gemm256d_persist(4096, 28672, 4096, 16 * 112) == 1
    assert L.gemm256d_persist(4096, 4096, 4096, 16 * 16) == 0
    L.gemm_persist_force(0)
    assert L.gemm256d_persist(4096, 28672, 4096, 16 * 112) == 0


@pytest.mark.parametrize("persist_mode", [0, 2])
@pytest.mark.parametrize("M,N,K", [(1000, 4096, 1024), (300, 2048, 4096)])
def test_wide_direct_epilogue_equals_staged(M, N, K, persist_mode):
    """The wide direct epilogue (permlane16 exchange + 16-B stores from the
    accumulators, common.h store_wide) writes the same bytes as the LDS-staged
    one at every tile height, one-tile and persistent: plain, residual in
    place with the fused statistic, SwiGLU with the fused norm scale."""
    L = ops.lib()
    torch.manual_seed(43)
    X = torch.randn(M, K, device=DEV).bfloat16()
    W = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    R = torch.randn(M, N, device=DEV).bfloat16()
    ss_in = (X.float().pow(2).sum(-1) * 0.5 * ref.SS_FIX).round().to(torch.int64)
    L.gemm_persist_force(persist_mode)
    try:
        for code in CODES:
            L.gemm_plan_set(N, K, [code] * 128)
            got = {}
            for wide in (0, 1):
                L.gemm_wide_force(wide)
                y = R.clone()
                ss = torch.zeros(M, dtype=torch.int64, device=DEV)
                ops.gemm(X, W, R=y, out=y, ss_out=ss)
                got[wide] = (ops.gemm(X, W), y, ss,
                             ops.gemm_silu(X, W, ss_in=ss_in, eps=1e-5))
            # outputs bitwise; the fused statistic up to fp32 summation order
            # (the wide epilogue sums a row's 128 columns in another order
            # before its one fixed-point add per wave)
            for a, b in zip(got[0][:2] + got[0][3:], got[1][:2] + got[1][3:]):
                assert torch.equal(a, b), code
            d = (got[0][2] - got[1][2]).abs().double() / got[0][2].double().clamp(min=1)
            assert d.max().item() < 1e-6, code
            assert rel_err(got[1][0], ref.gemm(X, W)) < 1e-2, code
            assert rel_err(got[1][3], ref.gemm_silu(X, W, ss_in=ss_in, eps=1e-5)) < 1e-2, code
    finally:
        L.gemm_wide_force(-1)
        L.gemm_persist_force(-1)
        L.gemm_plan_clear()
        ops._load_gemm_plan(L)
