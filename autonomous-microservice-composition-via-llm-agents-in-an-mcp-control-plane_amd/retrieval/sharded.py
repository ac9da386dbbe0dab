"""Corpus-sharded top-k cosine retrieval across the GPUs of a node (SURVEY
§2.6 K11 "corpus sharded per GPU", collective C6).

One MI355X holds ~10^8 x 1024 bf16 schema vectors in its 288 GB; beyond that
(or to cut per-query latency by N) every rank keeps a contiguous shard of the
corpus in its own HBM.  A query batch (replicated on every rank) is scored
against the local shard by the ``ops.topk_cosine`` HIP path, the local
(score, global id) top-k lists are all-gathered — k * 8 bytes per query per
rank, the only cross-GPU traffic — and every rank merges the N*k candidates
into the global top-k.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .. import ops


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, balanced [lo, hi) row range of rank ``rank``."""
    per, extra = divmod(n, world)
    lo = rank * per + min(rank, extra)
    return lo, lo + per + (1 if rank < extra else 0)


class ShardedIndex:
    def __init__(self, group=None, device="cpu"):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.device = torch.device(device)
        self.vectors: Optional[torch.Tensor] = None
        self.offset = 0
        self.total = 0

    def set_corpus(self, full_or_shard: torch.Tensor, total: Optional[int] = None,
                   offset: Optional[int] = None) -> None:
        """Either the full corpus (this rank keeps its slice) or, with
        ``total``/``offset``, an already-local shard."""
        if total is None:
            total = full_or_shard.shape[0]
            lo, hi = shard_range(total, self.rank, self.world)
            shard, offset = full_or_shard[lo:hi], lo
        else:
            shard = full_or_shard
        v = shard.to(self.device, torch.bfloat16)
        self.n_local = int(v.shape[0])
        if self.n_local % 4:                      # pad once here, never per query
            v = torch.cat([v, v.new_zeros(4 - self.n_local % 4, v.shape[1])])
        v = v.contiguous()
        self.vectors = ops.l2norm_rows(v) if v.shape[0] else v
        self.offset, self.total = int(offset), int(total)

    def search(self, queries: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """queries [B, D] (unit rows, same on every rank) -> global (scores [B, k] f32,
        ids [B, k] int64), identical on every rank."""
        q = queries.to(self.device, torch.bfloat16).contiguous()
        B = q.shape[0]
        k = min(k, self.total)
        kl = min(k, self.n_local)
        vals = torch.full((B, k), float("-inf"), device=self.device, dtype=torch.float32)
        ids = torch.full((B, k), -1, device=self.device, dtype=torch.int64)
        if kl > 0:
            v, i = ops.topk_cosine(q, self.vectors, kl, n_valid=self.n_local)
            vals[:, :kl] = v
            ids[:, :kl] = i.long() + self.offset
        if self.world == 1:
            return vals, ids
        gv = [torch.empty_like(vals) for _ in range(self.world)]
        gi = [torch.empty_like(ids) for _ in range(self.world)]
        dist.all_gather(gv, vals, group=self.group)
        dist.all_gather(gi, ids, group=self.group)
        allv, alli = torch.cat(gv, dim=1), torch.cat(gi, dim=1)
        top, pos = torch.topk(allv, k, dim=1)
        return top, torch.gather(alli, 1, pos)


def names_for(ids: torch.Tensor, names: Sequence[str]):
    return [[names[i] for i in row if 0 <= i < len(names)] for row in ids.tolist()]
