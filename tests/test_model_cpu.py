"""The paged, ragged, last-layer-row-restricted forward (models/llama.py) against
an independent dense fp32 Llama forward written here from the weights alone:
per sequence, full causal attention over its whole token history, no KV
cache, no paging, no fused epilogues.  A step that mixes a fresh prompt, a
continuation with cached context and a single-token decode checks the KV
write / read paths and that only the sampled rows are needed from the last
layer's MLP."""
import math

import numpy as np
import pytest
import torch

from mcp_amd.engine.batch import StepInputs, pack
from mcp_amd.engine.kv_cache import KVCache
from mcp_amd.models.llama import LlamaModel, get_config, random_weights
from mcp_amd.ops import reference as ref


def _dense_forward(cfg, w, ids):
    """fp32 hidden states after the final norm for every position of ONE sequence."""
    D, Hq, Hkv = cfg.head_dim, cfg.heads, cfg.kv_heads
    T = len(ids)
    cs = ref.rope_cos_sin(cfg.max_pos, D, cfg.rope_theta)
    pos = torch.arange(T)
    f = lambda t: t.float()
    x = f(w.embed)[torch.tensor(ids)]

    def norm(v, g):
        return v * torch.rsqrt(v.pow(2).mean(-1, keepdim=True) + cfg.eps) * f(g)

    def rope(v):                                   # [T, h, D], rotate-half
        c = cs[pos][..., 0].unsqueeze(1)
        s = cs[pos][..., 1].unsqueeze(1)
        a, b = v[..., : D // 2], v[..., D // 2:]
        return torch.cat([a * c - b * s, b * c + a * s], dim=-1)

    for lw in w.layers:
        h = norm(x, lw.attn_norm)
        qkv = (h @ f(lw.wqkv).t()).view(T, Hq + 2 * Hkv, D)
        q, k, v = rope(qkv[:, :Hq]), rope(qkv[:, Hq:Hq + Hkv]), qkv[:, Hq + Hkv:]
        k = k.repeat_interleave(Hq // Hkv, dim=1)
        v = v.repeat_interleave(Hq // Hkv, dim=1)
        S = torch.einsum("qhd,khd->hqk", q, k) / math.sqrt(D)
        S = S.masked_fill(torch.triu(torch.ones(T, T, dtype=torch.bool), 1), float("-inf"))
        a = torch.einsum("hqk,khd->qhd", torch.softmax(S, -1), v).reshape(T, Hq * D)
        x = x + a @ f(lw.wo).t()
        h = norm(x, lw.mlp_norm)
        g, u = ref.deinterleave_gate_up(f(lw.w_gate_up))
        x = x + (torch.nn.functional.silu(h @ g.t()) * (h @ u.t())) @ f(lw.w_down).t()
    return norm(x, w.final_norm)


@pytest.mark.parametrize("fused", ["1", "0"])
def test_paged_forward_matches_dense(fused, monkeypatch):
    """Non-trivial RMSNorm weights; ``fused`` = the fused-norm forward (norm
    weights folded into Wqkv / W_gate_up, row statistics from the residual
    GEMMs) or the standalone-RMSNorm forward, against the dense reference of
    the original (unfolded) weights."""
    import copy
    monkeypatch.setenv("MCP_FUSED_NORM", fused)
    torch.manual_seed(0)
    cfg = get_config("tiny")
    w = random_weights(cfg, "cpu", dtype=torch.float32, seed=11, std=0.05)
    g = torch.Generator().manual_seed(5)
    for lw in w.layers:
        lw.attn_norm.copy_(1 + 0.3 * torch.randn(lw.attn_norm.shape, generator=g))
        lw.mlp_norm.copy_(1 + 0.3 * torch.randn(lw.mlp_norm.shape, generator=g))
    w_ref = copy.deepcopy(w)                       # the model folds its weights in place
    model = LlamaModel(cfg, w, "cpu")
    assert model.fused_norm == (fused == "1")
    kv = KVCache(cfg.layers, cfg.kv_heads, cfg.head_dim, 16, "cpu", dtype=torch.float32)
    BS = 64
    rng = np.random.default_rng(1)
    # seq 0: 70-token prompt; seq 1: 40 cached tokens + 9 new; seq 2: 130 cached + 1 (decode)
    hist = [rng.integers(0, cfg.vocab_size, n).tolist() for n in (70, 49, 131)]
    cached = [0, 40, 130]
    blocks = [[0, 1], [2], [3, 4, 5]]
    # warm the caches of seqs 1 and 2 with a first step over their cached prefixes
    def step_for(chunks, starts, rows_last=True):
        ids, pos, slots, qs, ql, cl, rows = [], [], [], [], [], [], []
        for s, (toks, st) in enumerate(zip(chunks, starts)):
            qs.append(len(ids))
            for j, t in enumerate(toks):
                p = st + j
                ids.append(t)
                pos.append(p)
                slots.append(blocks[s][p // BS] * BS + p % BS)
            ql.append(len(toks))
            cl.append(st + len(toks))
            if toks and rows_last:
                rows.append(len(ids) - 1)
        bt = np.zeros((len(chunks), 3), np.int32)
        for s, b in enumerate(blocks):
            bt[s, :len(b)] = b
        return StepInputs(token_ids=np.asarray(ids, np.int32), positions=np.asarray(pos, np.int32),
                          slots=np.asarray(slots, np.int32), q_start=np.asarray(qs, np.int32),
                          q_len=np.asarray(ql, np.int32), ctx_len=np.asarray(cl, np.int32),
                          block_table=bt, logit_rows=np.asarray(rows, np.int32))
    warm = step_for([[], hist[1][:40], hist[2][:130]], [0, 0, 0], rows_last=False)
    out0 = model.forward(pack(warm, cfg.group, "cpu"), kv)
    assert out0.shape == (0, cfg.hidden)                     # no sampled rows: nothing returned
    step = step_for([hist[0], hist[1][40:], hist[2][130:]], cached)
    h = model.forward(pack(step, cfg.group, "cpu"), kv).float()
    assert h.shape == (3, cfg.hidden)
    for s in range(3):
        exp = _dense_forward(cfg, w_ref, hist[s])[-1]
        err = ((h[s] - exp).norm() / exp.norm()).item()
        assert err < 1e-4, (s, err)
