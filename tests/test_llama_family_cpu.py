"""Llama-3.1 family: rope scaling (128k context) in the host-built cos/sin
table, HF config.json round trip, and rejection of shapes the gfx950 kernels
do not serve.  The scaled frequencies are checked against transformers'
own ``llama3`` rope initialisation (installed here; no weights needed)."""
import json

import pytest
import torch

from mcp_amd.models.llama import CONFIGS, LlamaConfig, LlamaModel, random_weights
from mcp_amd.models.weights import config_from_hf, save_llama_safetensors
from mcp_amd.ops import reference as ref


def test_llama31_inv_freq_matches_transformers():
    tr = pytest.importorskip("transformers")
    from transformers.modeling_rope_utils import ROPE_INIT_FUNCTIONS
    cfg = tr.LlamaConfig(hidden_size=4096, num_attention_heads=32, num_key_value_heads=8,
                         rope_theta=500000.0, max_position_embeddings=131072,
                         rope_scaling={"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                       "high_freq_factor": 4.0,
                                       "original_max_position_embeddings": 8192})
    want, _ = ROPE_INIT_FUNCTIONS["llama3"](cfg, "cpu")
    got = ref.rope_inv_freq(128, 500000.0, CONFIGS["llama3.1-8b"].rope_scaling)
    torch.testing.assert_close(got.float(), want.float(), rtol=1e-6, atol=0)
    plain = ref.rope_inv_freq(128, 500000.0)
    assert torch.equal(got[:20], plain[:20])           # high frequencies untouched
    torch.testing.assert_close(got[-1], plain[-1] / 8)  # lowest frequency scaled by 1/factor


def test_llama31_cos_sin_table_and_positions_past_8k():
    cs = ref.rope_cos_sin(20000, 128, 500000.0, scaling=CONFIGS["llama3.1-8b"].rope_scaling)
    assert cs.shape == (20000, 64, 2)
    torch.testing.assert_close(cs[..., 0] ** 2 + cs[..., 1] ** 2, torch.ones(20000, 64))
    assert not torch.equal(cs, ref.rope_cos_sin(20000, 128, 500000.0))


def test_hf_config_roundtrip_with_rope_scaling(tmp_path):
    cfg = LlamaConfig("tiny31", hidden=256, layers=2, heads=2, kv_heads=1, ffn=512,
                      max_pos=16384, rope_scaling=(8.0, 1.0, 4.0, 8192))
    w = random_weights(cfg, "cpu", dtype=torch.float32, seed=1)
    save_llama_safetensors(cfg, w, tmp_path)
    c = json.loads((tmp_path / "config.json").read_text())
    assert c["rope_scaling"]["rope_type"] == "llama3"
    back = config_from_hf(tmp_path)
    assert back.rope_scaling == cfg.rope_scaling and back.max_pos == 16384
    m = LlamaModel(back, w, "cpu")
    torch.testing.assert_close(m.cos_sin, ref.rope_cos_sin(16384, 128, cfg.rope_theta,
                                                           scaling=cfg.rope_scaling))
    c["rope_scaling"] = {"rope_type": "yarn", "factor": 4.0}
    (tmp_path / "config.json").write_text(json.dumps(c))
    with pytest.raises(NotImplementedError):
        config_from_hf(tmp_path)


def test_unsupported_head_shapes_fail_loudly():
    # Llama-3.2-3B (24 q / 8 kv heads -> group 3) and -1B (head_dim 64)
    for cfg in (LlamaConfig("g3", hidden=384, layers=1, heads=3, kv_heads=1, ffn=512),
                LlamaConfig("d64", hidden=256, layers=1, heads=4, kv_heads=1, head_dim=64, ffn=512)):
        with pytest.raises(NotImplementedError):
            LlamaModel(cfg, None, "cpu")


# ---- GQA padding (Llama-3.2-3B: 24 q / 8 kv heads) --------------------------
def _one_sequence_forward(model, cfg, ids):
    import numpy as np
    from mcp_amd.engine.batch import StepInputs, pack
    from mcp_amd.engine.kv_cache import KVCache
    kv = KVCache(cfg.layers, cfg.kv_heads, cfg.head_dim, 4, "cpu", dtype=torch.float32)
    T = len(ids)
    step = StepInputs(token_ids=np.asarray(ids, np.int32), positions=np.arange(T, dtype=np.int32),
                      slots=np.arange(T, dtype=np.int32), q_start=np.asarray([0], np.int32),
                      q_len=np.asarray([T], np.int32), ctx_len=np.asarray([T], np.int32),
                      block_table=np.asarray([[0, 1]], np.int32),
                      logit_rows=np.asarray([T - 1], np.int32))
    return model.forward(pack(step, cfg.group, "cpu"), kv).float()[0]


def _unpadded(pc, w):
    from mcp_amd.models.llama import LayerWeights, LlamaWeights, unpad_o_cols, unpad_q_rows
    D = pc.head_dim
    layers = []
    for lw in w.layers:
        q, k, v = torch.split(lw.wqkv, [pc.heads * D, pc.kv_heads * D, pc.kv_heads * D])
        layers.append(LayerWeights(lw.attn_norm, torch.cat([unpad_q_rows(q, pc), k, v]),
                                   unpad_o_cols(lw.wo, pc), lw.mlp_norm, lw.w_gate_up, lw.w_down))
    return LlamaWeights(w.embed, layers, w.final_norm, w.lm_head)


def test_gqa_padding_is_exact_against_dense_unpadded_forward():
    import dataclasses
    from test_model_cpu import _dense_forward
    from mcp_amd.models.llama import pad_gqa
    cfg = LlamaConfig("g3", hidden=384, layers=2, heads=3, kv_heads=1, ffn=512, tie_embeddings=True)
    pc = pad_gqa(cfg)
    assert (pc.heads, pc.q_heads_true, pc.group, pc.group_true) == (4, 3, 4, 3)
    w = random_weights(pc, "cpu", dtype=torch.float32, seed=7, std=0.05)
    assert w.lm_head is w.embed
    ids = torch.randint(0, cfg.vocab_size, (90,), generator=torch.Generator().manual_seed(2)).tolist()
    got = _one_sequence_forward(LlamaModel(pc, w, "cpu"), pc, ids)
    want = _dense_forward(dataclasses.replace(cfg), _unpadded(pc, w), ids)[-1]
    assert ((got - want).norm() / want.norm()).item() < 1e-4


def test_gqa_padding_checkpoint_roundtrip(tmp_path):
    from mcp_amd.models.llama import pad_gqa
    from mcp_amd.models.weights import load_llama_safetensors
    pc = pad_gqa(LlamaConfig("g3", hidden=384, layers=2, heads=3, kv_heads=1, ffn=512,
                             tie_embeddings=True))
    w = random_weights(pc, "cpu", dtype=torch.float32, seed=3)
    save_llama_safetensors(pc, w, tmp_path)
    c = json.loads((tmp_path / "config.json").read_text())
    assert c["num_attention_heads"] == 3 and c["tie_word_embeddings"] is True
    cfg2, w2 = load_llama_safetensors(tmp_path, "cpu", dtype=torch.float32)
    assert (cfg2.heads, cfg2.q_heads_true, cfg2.tie_embeddings) == (4, 3, True)
    for a, b in zip(w.layers, w2.layers):
        assert torch.equal(a.wqkv, b.wqkv) and torch.equal(a.wo, b.wo)
    assert w2.lm_head is w2.embed
    # TP=2 is not possible with one kv head; shapes of the 3B config per rank at TP=8
    big = CONFIGS["llama3.2-3b"]
    assert big.group == 4 and big.group_true == 3 and abs(big.params() / 1e9 - 3.21) < 0.01
