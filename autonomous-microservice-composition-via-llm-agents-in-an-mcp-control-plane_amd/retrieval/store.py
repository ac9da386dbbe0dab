"""HBM-resident schema-embedding store + top-k cosine retrieval.

The reference keeps ``service_schemas(name, input_schema_vector)`` in
PostgreSQL/pgvector and has a fetch helper that is never called
(control_plane.py:46-55).  Here the vectors live in GPU memory
(bf16, unit-norm rows; 10^8 x 1024 fits in 288 GB) and retrieval is the
``ops.topk_cosine`` HIP path (MFMA scoring + segmented top-k).  It bounds the
planner prompt when the registry outgrows the context.

Embeddings: a deterministic signed feature-hashing embedder over word tokens
and character trigrams of the schema text (``ServiceRecord.schema_text``) and
of the intent.  It needs no model weights and gives lexical similarity, which
is what matching intents to service schemas needs without a trained encoder.
External vectors can be loaded with ``SchemaIndex.set_vectors``.
"""
from __future__ import annotations

import re
import zlib
from typing import List, Optional, Sequence

import numpy as np
import torch

from .. import ops

_WORD = re.compile(r"[a-z0-9]+")


def hash_embed(texts: Sequence[str], dim: int = 1024) -> np.ndarray:
    out = np.zeros((len(texts), dim), np.float32)
    for r, t in enumerate(texts):
        t = t.lower().replace("_", " ").replace("-", " ")
        feats = _WORD.findall(t)
        grams = []
        for w in feats:
            ww = f"#{w}#"
            grams += [ww[i:i + 3] for i in range(len(ww) - 2)]
        for f, wgt in [(x, 1.0) for x in feats] + [(g, 0.5) for g in grams]:
            h = zlib.crc32(f.encode())
            out[r, h % dim] += wgt if (h >> 31) & 1 else -wgt
    n = np.linalg.norm(out, axis=1, keepdims=True)
    return out / np.maximum(n, 1e-12)


class SchemaIndex:
    def __init__(self, registry=None, dim: int = 1024, device="cpu"):
        self.registry = registry
        self.dim = dim
        self.device = torch.device(device)
        self._version = None
        self.names: List[str] = []
        self.vectors: Optional[torch.Tensor] = None     # [N, dim] bf16, unit rows

    def set_vectors(self, names: Sequence[str], vectors) -> None:
        """Upload and normalise the corpus once.  Rows are padded to a multiple
        of 4 here (zero rows, never returned: ``n_valid``) so no query ever
        copies the corpus (the unfused scoring GEMM writes 16-B column groups)."""
        v = torch.as_tensor(vectors).to(self.device, torch.bfloat16)
        n = v.shape[0]
        if n % 4:
            v = torch.cat([v, v.new_zeros(4 - n % 4, v.shape[1])])
        v = v.contiguous()
        ops.l2norm_rows(v)
        self.names, self.vectors = list(names), v

    def refresh(self, services: Optional[Sequence[dict]] = None) -> None:
        ver = getattr(self.registry, "version", None)
        if services is None:
            if self.vectors is not None and ver == self._version:
                return
            services = self.registry.list_services()
        texts = [s.schema_text() if hasattr(s, "schema_text") else str(s) for s in services]
        self.set_vectors([s["name"] for s in services], hash_embed(texts, self.dim))
        self._version = ver

    def embed_queries(self, intents: Sequence[str]) -> torch.Tensor:
        q = torch.from_numpy(hash_embed(intents, self.dim)).to(self.device, torch.bfloat16)
        return ops.l2norm_rows(q.contiguous())

    def search_names(self, intents: Sequence[str], k: int):
        vals, idx = ops.topk_cosine(self.embed_queries(intents), self.vectors, k,
                                    n_valid=len(self.names))
        idx = idx.cpu().tolist()
        return [[self.names[i] for i in row if 0 <= i < len(self.names)] for row in idx], vals.cpu()

    def search(self, intent: str, k: int, services: Sequence[dict]) -> List[dict]:
        if self.vectors is None or len(self.names) != len(services) or \
                getattr(self.registry, "version", None) != self._version:
            self.refresh(services)
        names, _ = self.search_names([intent], k)
        by = {s["name"]: s for s in services}
        return [by[n] for n in names[0] if n in by]
