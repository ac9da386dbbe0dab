"""Plain-PyTorch fp32 reference implementations of every HIP kernel.

These define the semantics the gfx950 kernels are tested against
(tests/test_kernels_gpu.py) and run the model on CPU in the CPU test tier.
They are never used for GPU tensors: ``ops`` routes GPU tensors to the HIP
library and raises if it is missing.
"""
from __future__ import annotations

import math
from typing import Optional

import torch


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    inv = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (xf * inv * w.float()).to(x.dtype)


def add_rmsnorm(x, residual, w, eps):
    residual.copy_((x.float() + residual.float()).to(residual.dtype))
    return rmsnorm(residual, w, eps)


def silu_mul(x: torch.Tensor) -> torch.Tensor:
    F = x.shape[-1] // 2
    g, u = x[..., :F].float(), x[..., F:].float()
    return (torch.nn.functional.silu(g) * u).to(x.dtype)


GU_GROUP = 16   # gate/up row interleave granularity of the fused SwiGLU GEMM


def interleave_gate_up(g: torch.Tensor, u: torch.Tensor) -> torch.Tensor:
    """[F, H] gate + [F, H] up -> [2F, H] rows [g0..g15, u0..u15, g16..g31, ...]."""
    F, H = g.shape
    return torch.stack([g.view(F // GU_GROUP, GU_GROUP, H), u.view(F // GU_GROUP, GU_GROUP, H)],
                       dim=1).reshape(2 * F, H)


def deinterleave_gate_up(w: torch.Tensor):
    F2, H = w.shape
    v = w.view(F2 // (2 * GU_GROUP), 2, GU_GROUP, H)
    return v[:, 0].reshape(F2 // 2, H), v[:, 1].reshape(F2 // 2, H)


SS_FIX = float(1 << 20)         # fixed-point unit of the fused-norm row statistics (csrc/common.h)


def row_sumsq(x: torch.Tensor) -> torch.Tensor:
    """Per-row sum of squares of a bf16 [T, H] matrix as int64 fixed point."""
    return torch.round(x.float().pow(2).sum(-1) * SS_FIX).to(torch.int64)


def norm_row_scale(ss: torch.Tensor, H: int, eps: float) -> torch.Tensor:
    """[T, 1] fp32 rsqrt(mean(x^2) + eps) from fixed-point row statistics."""
    return torch.rsqrt(ss.double().div(SS_FIX).float() / H + eps).unsqueeze(-1)


def gemm_silu(X, W_interleaved, ss_in=None, eps: float = 0.0):
    y = (X.float() @ W_interleaved.float().t())
    if ss_in is not None:                      # fused RMSNorm: rows scaled after the GEMM
        y = y * norm_row_scale(ss_in[:X.shape[0]], X.shape[-1], eps)
    T, F2 = y.shape
    y = y.view(T, F2 // (2 * GU_GROUP), 2, GU_GROUP)
    g, u = y[:, :, 0], y[:, :, 1]
    return (torch.nn.functional.silu(g) * u).reshape(T, F2 // 2).to(X.dtype)


def gemm(X, W, R: Optional[torch.Tensor] = None):
    y = X.float() @ W.float().t()
    if R is not None:
        y = y + R.float()
    return y.to(X.dtype)


def rope_inv_freq(head_dim: int, theta: float, scaling=None) -> torch.Tensor:
    """Rotary inverse frequencies [D/2] (fp64).  ``scaling`` = (factor,
    low_freq_factor, high_freq_factor, original_max_pos) applies Llama-3.1's
    frequency-dependent rescaling: wavelengths longer than
    original_max_pos / low_freq_factor are divided by ``factor``, shorter than
    original_max_pos / high_freq_factor are kept, and the band in between is
    interpolated linearly in 1/wavelength."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling is None:
        return inv
    factor, lo, hi, orig = scaling
    wavelen = 2 * math.pi / inv
    smooth = (orig / wavelen - lo) / (hi - lo)
    mid = (1 - smooth) * inv / factor + smooth * inv
    return torch.where(wavelen > orig / lo, inv / factor, torch.where(wavelen < orig / hi, inv, mid))


def rope_cos_sin(max_pos: int, head_dim: int, theta: float, device=None,
                 scaling=None) -> torch.Tensor:
    inv = rope_inv_freq(head_dim, theta, scaling)
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    cs = torch.stack([f.cos(), f.sin()], dim=-1).float()      # [P, D/2, 2]
    return cs.to(device) if device is not None else cs


def apply_rope(x: torch.Tensor, pos: torch.Tensor, cos_sin: torch.Tensor) -> torch.Tensor:
    """x: [T, H, D]; rotate-half convention."""
    D = x.shape[-1]
    cs = cos_sin[pos.long()]                                    # [T, D/2, 2]
    c, s = cs[..., 0].unsqueeze(1), cs[..., 1].unsqueeze(1)
    xf = x.float()
    a, b = xf[..., : D // 2], xf[..., D // 2:]
    return torch.cat([a * c - b * s, b * c + a * s], dim=-1).to(x.dtype)


def rope_kv(qkv, pos, slots, cos_sin, q_out, k_cache, v_cache, Hq, Hkv, D):
    T = pos.numel()
    x = qkv.view(T, Hq + 2 * Hkv, D)
    q, k, v = x[:, :Hq], x[:, Hq:Hq + Hkv], x[:, Hq + Hkv:]
    q_out.view(T, Hq, D).copy_(apply_rope(q, pos, cos_sin))
    kr = apply_rope(k, pos, cos_sin)
    BS = k_cache.shape[2]
    for t in range(T):
        s = int(slots[t])
        if s < 0:
            continue
        b, o = s // BS, s % BS
        k_cache[b, :, o] = kr[t]
        v_cache[b, :, o] = v[t]


def paged_attention(q, k_cache, v_cache, q_start, q_len, ctx_len, block_table, scale):
    """q: [T, Hq, D]; caches [nb, Hkv, BS, D]; causal over each sequence's context."""
    T, Hq, D = q.shape
    Hkv, BS = k_cache.shape[1], k_cache.shape[2]
    G = Hq // Hkv
    out = torch.zeros_like(q)
    for s in range(q_start.numel()):
        qs, ql, cl = int(q_start[s]), int(q_len[s]), int(ctx_len[s])
        if ql == 0:
            continue
        nblk = (cl + BS - 1) // BS
        blocks = block_table[s, :nblk].long()
        K = k_cache[blocks].permute(1, 0, 2, 3).reshape(Hkv, nblk * BS, D)[:, :cl].float()
        V = v_cache[blocks].permute(1, 0, 2, 3).reshape(Hkv, nblk * BS, D)[:, :cl].float()
        K = K.repeat_interleave(G, dim=0)
        V = V.repeat_interleave(G, dim=0)
        Q = q[qs:qs + ql].float().transpose(0, 1)                 # [Hq, ql, D]
        S = Q @ K.transpose(1, 2) * scale                         # [Hq, ql, cl]
        qpos = torch.arange(cl - ql, cl).unsqueeze(1)
        kpos = torch.arange(cl).unsqueeze(0)
        S = S.masked_fill(kpos > qpos, float("-inf"))
        P = torch.softmax(S, dim=-1)
        out[qs:qs + ql] = (P @ V).transpose(0, 1).to(q.dtype)
    return out


def sample_allowed_logits(hidden, W, allow_ptr, allow_ids):
    """Returns the list of (ids, logits) per row: the exact quantities the fused
    kernel draws from."""
    out = []
    for s in range(hidden.shape[0]):
        ids = allow_ids[int(allow_ptr[s]):int(allow_ptr[s + 1])].long()
        out.append((ids, (W[ids].float() @ hidden[s].float())))
    return out


def topk_cosine(queries: torch.Tensor, corpus: torch.Tensor, k: int):
    qn = torch.nn.functional.normalize(queries.float(), dim=-1)
    cn = torch.nn.functional.normalize(corpus.float(), dim=-1)
    return torch.topk(qn @ cn.t(), k=min(k, corpus.shape[0]), dim=-1)


def attention_scale(head_dim: int) -> float:
    return 1.0 / math.sqrt(head_dim)
