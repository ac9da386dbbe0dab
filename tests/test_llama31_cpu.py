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
