"""Hugging Face Llama-3 safetensors <-> engine weight layout (SURVEY §2.6,
"TP weight sharder and random-init / safetensors loader").

The engine's layout differs from the HF checkpoint in two fused tensors:

* ``wqkv``      = cat(q_proj, k_proj, v_proj) rows (one GEMM, K1);
* ``w_gate_up`` = gate_proj / up_proj rows interleaved in 16-row groups so the
  SwiGLU epilogue of the GEMM finds each gate row next to its up row (K7 fused
  into K1, ``ops.reference.interleave_gate_up``).

Tensor-parallel loading reads only this rank's shard of every sharded tensor
(``safe_open(...).get_slice``), so a 70B checkpoint is never materialised in
full on any rank: q/k/v and gate/up are split by rows (whole heads / FFN
columns), o_proj and down_proj by columns, norms / embeddings / LM head are
replicated (Megatron 1-D, ``models.llama``).

HF Llama checkpoints already store q/k in the rotate-half RoPE convention the
``rope_kv`` kernel implements; Meta's original ``consolidated.*.pth`` (interleaved
RoPE, pickled) are not supported (and would need a non-weights-only loader).
Only safetensors are read: they execute nothing from the file.
"""
from __future__ import annotations

import json
import os
from pathlib import Path
from typing import Dict, List, Optional

import torch

from ..ops import reference as ref
from .llama import (LayerWeights, LlamaConfig, LlamaWeights, pad_gqa, pad_o_cols, pad_q_rows,
                    shard_cols, shard_rows, unpad_o_cols, unpad_q_rows)


def config_from_hf(path) -> LlamaConfig:
    """``config.json`` of an HF Llama checkpoint -> LlamaConfig."""
    c = json.loads((Path(path) / "config.json").read_text())
    heads = c["num_attention_heads"]
    rs = c.get("rope_scaling") or None
    scaling = None
    if rs is not None:
        kind = rs.get("rope_type", rs.get("type"))
        if kind != "llama3":
            raise NotImplementedError(f"rope_scaling type {kind!r} (supported: llama3)")
        scaling = (float(rs["factor"]), float(rs.get("low_freq_factor", 1.0)),
                   float(rs.get("high_freq_factor", 4.0)),
                   int(rs.get("original_max_position_embeddings", 8192)))
    return pad_gqa(LlamaConfig(
        name=c.get("_name_or_path") or Path(path).name,
        vocab_size=c["vocab_size"], hidden=c["hidden_size"], layers=c["num_hidden_layers"],
        heads=heads, kv_heads=c.get("num_key_value_heads", heads),
        head_dim=c.get("head_dim") or c["hidden_size"] // heads, ffn=c["intermediate_size"],
        rope_theta=float(c.get("rope_theta", 10000.0)), eps=float(c.get("rms_norm_eps", 1e-5)),
        max_pos=int(c.get("max_position_embeddings", 8192)), rope_scaling=scaling,
        tie_embeddings=bool(c.get("tie_word_embeddings", False))))


def _tensor_index(path: Path) -> Dict[str, Path]:
    """tensor name -> shard file (sharded index or a single model.safetensors)."""
    idx = path / "model.safetensors.index.json"
    if idx.exists():
        wm = json.loads(idx.read_text())["weight_map"]
        return {k: path / v for k, v in wm.items()}
    files = sorted(path.glob("*.safetensors"))
    if not files:
        raise FileNotFoundError(f"no safetensors under {path}")
    from safetensors import safe_open
    out = {}
    for f in files:
        with safe_open(str(f), framework="pt", device="cpu") as h:
            for k in h.keys():
                out[k] = f
    return out


class _Reader:
    def __init__(self, path: Path):
        from safetensors import safe_open
        self._open = safe_open
        self.index = _tensor_index(path)
        self._handles = {}

    def _h(self, name):
        f = self.index[name]
        h = self._handles.get(f)
        if h is None:
            h = self._open(str(f), framework="pt", device="cpu")
            self._handles[f] = h
        return h

    def has(self, name) -> bool:
        return name in self.index

    def full(self, name) -> torch.Tensor:
        return self._h(name).get_tensor(name)

    def rows(self, name, rank, tp) -> torch.Tensor:
        sl = self._h(name).get_slice(name)
        n = sl.get_shape()[0] // tp
        return sl[rank * n:(rank + 1) * n]

    def cols(self, name, rank, tp) -> torch.Tensor:
        sl = self._h(name).get_slice(name)
        n = sl.get_shape()[1] // tp
        return sl[:, rank * n:(rank + 1) * n]


def load_llama_safetensors(path, device, cfg: Optional[LlamaConfig] = None, tp_rank: int = 0,
                           tp: int = 1, dtype=torch.bfloat16):
    """Returns (cfg, LlamaWeights) for this TP rank, tensors on ``device``."""
    path = Path(path)
    cfg = cfg or config_from_hf(path)
    r = _Reader(path)
    dev = torch.device(device)

    def put(t):
        return t.to(dtype).contiguous().to(dev)

    layers: List[LayerWeights] = []
    for i in range(cfg.layers):
        p = f"model.layers.{i}."
        if cfg.q_heads_true:       # GQA padding happens on the full tensor, then the TP split
            q = shard_rows(pad_q_rows(r.full(p + "self_attn.q_proj.weight"), cfg), tp_rank, tp)
            o = shard_cols(pad_o_cols(r.full(p + "self_attn.o_proj.weight"), cfg), tp_rank, tp)
        else:
            q = r.rows(p + "self_attn.q_proj.weight", tp_rank, tp)
            o = r.cols(p + "self_attn.o_proj.weight", tp_rank, tp)
        k = r.rows(p + "self_attn.k_proj.weight", tp_rank, tp)
        v = r.rows(p + "self_attn.v_proj.weight", tp_rank, tp)
        g = r.rows(p + "mlp.gate_proj.weight", tp_rank, tp)
        u = r.rows(p + "mlp.up_proj.weight", tp_rank, tp)
        layers.append(LayerWeights(
            attn_norm=put(r.full(p + "input_layernorm.weight")),
            wqkv=put(torch.cat([q, k, v])),
            wo=put(o),
            mlp_norm=put(r.full(p + "post_attention_layernorm.weight")),
            w_gate_up=put(ref.interleave_gate_up(g, u)),
            w_down=put(r.cols(p + "mlp.down_proj.weight", tp_rank, tp))))
    embed = put(r.full("model.embed_tokens.weight"))
    lm = put(r.full("lm_head.weight")) if r.has("lm_head.weight") else embed   # tied embeddings
    return cfg, LlamaWeights(embed=embed, layers=layers, final_norm=put(r.full("model.norm.weight")),
                             lm_head=lm)


def save_llama_safetensors(cfg: LlamaConfig, w: LlamaWeights, path, shard_layers: int = 0) -> None:
    """Write TP=1 engine weights as an HF-layout checkpoint (config.json +
    safetensors, optionally sharded by layer count with an index)."""
    from safetensors.torch import save_file
    path = Path(path)
    path.mkdir(parents=True, exist_ok=True)
    D = cfg.head_dim
    tensors: Dict[str, torch.Tensor] = {}
    for i, lw in enumerate(w.layers):
        p = f"model.layers.{i}."
        q, k, v = torch.split(lw.wqkv, [cfg.heads * D, cfg.kv_heads * D, cfg.kv_heads * D])
        q = unpad_q_rows(q, cfg)
        g, u = ref.deinterleave_gate_up(lw.w_gate_up)
        tensors.update({
            p + "input_layernorm.weight": lw.attn_norm, p + "self_attn.q_proj.weight": q,
            p + "self_attn.k_proj.weight": k, p + "self_attn.v_proj.weight": v,
            p + "self_attn.o_proj.weight": unpad_o_cols(lw.wo, cfg), p + "post_attention_layernorm.weight": lw.mlp_norm,
            p + "mlp.gate_proj.weight": g, p + "mlp.up_proj.weight": u,
            p + "mlp.down_proj.weight": lw.w_down})
    tensors["model.embed_tokens.weight"] = w.embed
    tensors["model.norm.weight"] = w.final_norm
    if not cfg.tie_embeddings:
        tensors["lm_head.weight"] = w.lm_head
    tensors = {k: t.detach().cpu().contiguous() for k, t in tensors.items()}
    if shard_layers <= 0:
        save_file(tensors, str(path / "model.safetensors"))
    else:
        weight_map, shards = {}, {}
        for k in tensors:
            li = int(k.split(".")[2]) // shard_layers if k.startswith("model.layers.") else -1
            shards.setdefault(li, []).append(k)
        n = len(shards)
        for j, li in enumerate(sorted(shards)):
            fn = f"model-{j + 1:05d}-of-{n:05d}.safetensors"
            save_file({k: tensors[k] for k in shards[li]}, str(path / fn))
            weight_map.update({k: fn for k in shards[li]})
        (path / "model.safetensors.index.json").write_text(
            json.dumps({"metadata": {}, "weight_map": weight_map}, indent=1))
    (path / "config.json").write_text(json.dumps({
        "architectures": ["LlamaForCausalLM"], "model_type": "llama", "_name_or_path": cfg.name,
        "vocab_size": cfg.vocab_size, "hidden_size": cfg.hidden, "num_hidden_layers": cfg.layers,
        "num_attention_heads": cfg.q_heads_true or cfg.heads, "num_key_value_heads": cfg.kv_heads,
        "head_dim": D, "tie_word_embeddings": cfg.tie_embeddings,
        "intermediate_size": cfg.ffn, "rope_theta": cfg.rope_theta, "rms_norm_eps": cfg.eps,
        "max_position_embeddings": cfg.max_pos, "torch_dtype": "bfloat16",
        **({"rope_scaling": {"rope_type": "llama3", "factor": cfg.rope_scaling[0],
                             "low_freq_factor": cfg.rope_scaling[1],
                             "high_freq_factor": cfg.rope_scaling[2],
                             "original_max_position_embeddings": cfg.rope_scaling[3]}}
           if cfg.rope_scaling else {})}, indent=1))


def model_from_checkpoint(path, device, tp_rank: int = 0, tp: int = 1, tp_group=None):
    """LlamaModel over an HF safetensors checkpoint directory."""
    from .llama import LlamaModel
    cfg, w = load_llama_safetensors(path, device, tp_rank=tp_rank, tp=tp)
    return LlamaModel(cfg, w, device, tp_rank, tp, tp_group)


def checkpoint_dir_from_env() -> Optional[str]:
    p = os.environ.get("MCP_CHECKPOINT")
    return p if p and Path(p).is_dir() else None
