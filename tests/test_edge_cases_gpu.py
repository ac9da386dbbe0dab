"""Edge cases on the MI355X:

* NaN propagation: a NaN input must give NaN exactly where the fp32 reference
  does, through every GEMM path the tile plan picks (skinny / split-K / 256d /
  hybrid tail, chosen by M), the SwiGLU epilogue and RMSNorm.  The bf16
  conversions are plain casts (``v_cvt_pk_bf16_f32``), not bit tricks that
  turn NaN into Inf (``MICROARCH:464``).
* Prefill / decode consistency of the paged KV cache on the HIP kernels: the
  hidden state of token t is the same whether t arrives in one prefill step, as
  a decode step after a 130-token prefill, or after chunked prefills that
  cross a 64-token block boundary.
"""
import math

import numpy as np
import pytest
import torch

import mcp_amd.ops as ops
from mcp_amd.engine.batch import StepInputs, pack
from mcp_amd.engine.kv_cache import KVCache
from mcp_amd.models.llama import LlamaModel, get_config, random_weights
from mcp_amd.ops import reference as ref

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")]

DEV = "cuda"


@pytest.mark.parametrize("M", [1, 40, 300, 2600])
def test_gemm_nan_propagation(M):
    torch.manual_seed(5)
    K, N = 4096, 4096
    X = torch.randn(M, K, device=DEV).bfloat16()
    X[M // 2, 7] = float("nan")
    W = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    Y = ops.gemm(X, W)
    exp = ref.gemm(X, W).float()
    assert torch.equal(torch.isnan(Y.float()), torch.isnan(exp))
    assert torch.isnan(Y[M // 2]).all()
    ok = ~torch.isnan(exp)
    assert torch.isfinite(Y.float()[ok]).all()


@pytest.mark.parametrize("M", [3, 520])
def test_swiglu_and_rmsnorm_nan_propagation(M):
    torch.manual_seed(6)
    K, F = 1024, 3584
    X = torch.randn(M, K, device=DEV).bfloat16()
    X[M - 1, 3] = float("nan")
    g = (torch.randn(F, K, device=DEV) / math.sqrt(K)).bfloat16()
    u = (torch.randn(F, K, device=DEV) / math.sqrt(K)).bfloat16()
    y = ops.gemm_silu(X, ref.interleave_gate_up(g, u).contiguous()).float()
    assert torch.isnan(y[M - 1]).all()
    assert torch.isfinite(y[:M - 1]).all()
    w = (torch.rand(K, device=DEV) + 0.5).bfloat16()
    n = ops.rmsnorm(X, w, 1e-5).float()
    assert torch.equal(torch.isnan(n), torch.isnan(ref.rmsnorm(X, w, 1e-5).float()))
    assert torch.isnan(n[M - 1]).all() and torch.isfinite(n[:M - 1]).all()


def _step(chunks, starts, blocks, BS=64):
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
        rows.append(len(ids) - 1)
    bt = np.zeros((len(chunks), max(len(b) for b in blocks)), np.int32)
    for s, b in enumerate(blocks):
        bt[s, :len(b)] = b
    return StepInputs(token_ids=np.asarray(ids, np.int32), positions=np.asarray(pos, np.int32),
                      slots=np.asarray(slots, np.int32), q_start=np.asarray(qs, np.int32),
                      q_len=np.asarray(ql, np.int32), ctx_len=np.asarray(cl, np.int32),
                      block_table=bt, logit_rows=np.asarray(rows, np.int32))


def test_prefill_decode_consistency_on_hip_kernels():
    cfg = get_config("tiny")
    model = LlamaModel(cfg, random_weights(cfg, DEV, seed=21), DEV)
    toks = np.random.default_rng(4).integers(0, cfg.vocab_size, 131).tolist()
    blocks = [[5, 2, 7]]                    # non-contiguous physical blocks

    def run(splits):
        kv = KVCache(cfg.layers, cfg.kv_heads, cfg.head_dim, 8, DEV)
        h, start = None, 0
        for n in splits:
            h = model.forward(pack(_step([toks[start:start + n]], [start], blocks), cfg.group, DEV),
                              kv)
            start += n
        torch.cuda.synchronize()
        return h.float()

    one = run([131])                         # whole prompt in one prefill
    dec = run([130, 1])                      # prefill, then one decode step
    chunked = run([64, 66, 1])               # chunked prefill across a block edge
    assert torch.isfinite(one).all()
    for h in (dec, chunked):
        err = ((h - one).norm() / one.norm()).item()
        assert err < 2e-2, err
