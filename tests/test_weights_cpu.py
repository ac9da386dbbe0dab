"""safetensors checkpoint round trip and TP-sharded loading (CPU)."""
import torch

from mcp_amd.engine.engine import LLMEngine
from mcp_amd.models.llama import LlamaModel, get_config, random_weights, shard_layer
from mcp_amd.models.weights import config_from_hf, load_llama_safetensors, save_llama_safetensors


def test_safetensors_roundtrip_forward(tmp_path):
    cfg = get_config("tiny")
    w = random_weights(cfg, "cpu", seed=3)
    save_llama_safetensors(cfg, w, tmp_path / "ck")
    cfg2 = config_from_hf(tmp_path / "ck")
    assert (cfg2.hidden, cfg2.layers, cfg2.heads, cfg2.kv_heads, cfg2.ffn) == \
        (cfg.hidden, cfg.layers, cfg.heads, cfg.kv_heads, cfg.ffn)
    _, w2 = load_llama_safetensors(tmp_path / "ck", "cpu", cfg=cfg)
    for a, b in zip(w.layers, w2.layers):
        for f in ("wqkv", "wo", "w_gate_up", "w_down", "attn_norm", "mlp_norm"):
            assert torch.equal(getattr(a, f), getattr(b, f)), f
    assert torch.equal(w.embed, w2.embed) and torch.equal(w.lm_head, w2.lm_head)
    # identical greedy generations
    outs = []
    for ww in (w, w2):
        eng = LLMEngine(LlamaModel(cfg, ww, "cpu"), num_blocks=32, max_batch=4, temperature=0.0)
        from mcp_amd.planner.grammar import DagDecoder, GrammarSpec
        from mcp_amd.planner.tokenizer import get_tokenizer
        from mcp_amd.registry import synthetic_registry
        spec = GrammarSpec(synthetic_registry(4, seed=1), get_tokenizer(), max_nodes=2)
        seq = eng.submit(DagDecoder(spec), [1, 2, 3, 4, 5])
        eng.run()
        outs.append(seq.result)
    assert outs[0] == outs[1]


def test_sharded_checkpoint_tp_slices(tmp_path):
    cfg = get_config("tiny-tp")
    w = random_weights(cfg, "cpu", seed=5)
    save_llama_safetensors(cfg, w, tmp_path / "ck", shard_layers=1)
    assert (tmp_path / "ck" / "model.safetensors.index.json").exists()
    for rank in range(2):
        _, ws = load_llama_safetensors(tmp_path / "ck", "cpu", cfg=cfg, tp_rank=rank, tp=2)
        for full, got in zip(w.layers, ws.layers):
            exp = shard_layer(full, cfg, rank, 2)
            for f in ("wqkv", "wo", "w_gate_up", "w_down"):
                assert torch.equal(getattr(exp, f), getattr(got, f)), (rank, f)
