"""hipGraph capture of small engine steps (SURVEY §2.6 "hipGraph bucket
capture", BASELINE config 5: continuous-batching decode, hipGraph).

A small step (a few concurrent requests, a decode / jump-forward span each)
costs ~2.5 ms of weight streaming on the GPU but ~260 kernel launches
(32 layers x 8 ops + sampling); issued one by one from Python the launches,
not the GPU, set the step time.  Steps with at most ``max(BUCKETS)`` tokens are
therefore replayed from a captured hipGraph (``torch.cuda.CUDAGraph`` is the
HIP graph API on ROCm):

* every step of a bucket uses ONE fixed int32 layout (``pack_static``):
  tokens padded to the bucket size (padding writes no KV: slot -1), sequence
  arrays padded with empty dummy sequences, attention work lists padded with
  work items of an empty sequence (the kernel's early exit), a block table of
  fixed width, grammar-allowed sets padded to empty rows;
* the per-step H2D copy lands in the bucket's static device buffer, then the
  graph replays forward + fused LM-head/grammar/sampling (K9) and leaves the
  tokens in a static output;
* the sampler's RNG counter (request uid, sample index) travels in the
  buffer and the seed is constant, so nothing in the graph changes per step.

Cascade attention and KV copy-on-write are eager-only: a step that needs them
(a large batch sharing a prefix, or a request just attached to its prefix)
runs eagerly.  The capture happens lazily on first use of a bucket, after one
eager warm-up of the same static step.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional

import numpy as np
import torch

from .. import ops
from .batch import BLOCK_SIZE, HostStager, StepInputs, build_work, tokens_per_item, views

BUCKETS = (16, 32, 64, 128, 256)
ALLOWED_PER_ROW = 64


@dataclasses.dataclass
class _Bucket:
    size: int
    sizes: List[int]
    S: int
    buf: torch.Tensor
    graph: object = None
    tokens: Optional[torch.Tensor] = None
    dstep: object = None


class GraphRunner:
    def __init__(self, model, kv, temperature: float, seed: int, buckets=BUCKETS):
        self.model, self.kv = model, kv
        self.device = model.device
        self.group = model.cfg.group
        self.mblk = (model.cfg.max_pos + BLOCK_SIZE - 1) // BLOCK_SIZE
        self.temperature, self.seed = float(temperature), int(seed)
        self.buckets = tuple(sorted(buckets))
        self._b: Dict[int, _Bucket] = {}
        self._pool = None
        self.stager = HostStager(self.device)
        self.replays = 0

    # ---------------------------------------------------------------- layout
    def _caps(self, b: int):
        t1 = tokens_per_item(1, self.group)
        t4 = tokens_per_item(4, self.group)
        S = b + 1                          # >= one empty dummy sequence
        cap1 = b
        cap4 = b // t4 + b // (2 * t1) + 1
        return S, cap1, cap4, S * ALLOWED_PER_ROW

    def _sizes(self, b: int) -> List[int]:
        S, cap1, cap4, A = self._caps(b)
        # same part order as batch.pack_host / views
        return [b, b, b, S, S, S, S, S * self.mblk, cap1, cap1, cap4, cap4, 0, 0, 0, 0,
                S + 1, A, S]

    def bucket_for(self, step: StepInputs) -> Optional[int]:
        T = step.num_tokens
        S = int(step.q_len.shape[0])
        A = int(step.allow_ids.shape[0]) if step.allow_ids is not None else 0
        if step.block_table.shape[1] > self.mblk:
            return None
        for b in self.buckets:
            Sb, _, _, Acap = self._caps(b)
            if T <= b and S < Sb and A <= Acap:
                return b
        return None

    def pack_static(self, step: Optional[StepInputs], b: int) -> Optional[np.ndarray]:
        S_b, cap1, cap4, A_cap = self._caps(b)
        T = step.num_tokens if step is not None else 0
        S = int(step.q_len.shape[0]) if step is not None else 0
        ids = np.zeros(b, np.int32)
        pos = np.zeros(b, np.int32)
        slots = np.full(b, -1, np.int32)
        rows = np.zeros(S_b, np.int32)
        qs, ql, cl = (np.zeros(S_b, np.int32) for _ in range(3))
        bt = np.zeros((S_b, self.mblk), np.int32)
        ws1 = np.full(cap1, S_b - 1, np.int32)
        wq1 = np.zeros(cap1, np.int32)
        ws4 = np.full(cap4, S_b - 1, np.int32)
        wq4 = np.zeros(cap4, np.int32)
        aptr = np.zeros(S_b + 1, np.int32)
        aids = np.zeros(A_cap, np.int32)
        ctr = np.zeros(S_b, np.int32)
        if step is not None:
            ids[:T], pos[:T], slots[:T] = step.token_ids, step.positions, step.slots
            R = int(step.logit_rows.shape[0])
            rows[:R] = step.logit_rows
            qs[:S], ql[:S], cl[:S] = step.q_start, step.q_len, step.ctx_len
            bt[:S, :step.block_table.shape[1]] = step.block_table
            work = build_work(step.q_len.tolist(), self.group)
            if len(work[1][0]) > cap1 or len(work[4][0]) > cap4:
                return None
            ws1[:len(work[1][0])], wq1[:len(work[1][1])] = work[1][0], work[1][1]
            ws4[:len(work[4][0])], wq4[:len(work[4][1])] = work[4][0], work[4][1]
            if R:
                aptr[:R + 1] = step.allow_ptr
                aptr[R + 1:] = step.allow_ptr[-1]
                A = int(step.allow_ids.shape[0])
                if A > A_cap:
                    return None
                aids[:A] = step.allow_ids
                ctr[:R] = step.sample_ctr
        z = np.zeros(0, np.int32)
        return np.concatenate([ids, pos, slots, rows, qs, ql, cl, bt.reshape(-1), ws1, wq1, ws4,
                               wq4, z, z, z, z, aptr, aids, ctr])

    # ---------------------------------------------------------------- graphs
    def _body(self, e: _Bucket):
        hidden = self.model.forward(e.dstep, self.kv)
        return ops.sample_allowed(hidden, self.model.w.lm_head, e.dstep.allow_ptr,
                                  e.dstep.allow_ids, e.dstep.sample_ctr, self.temperature,
                                  self.seed)

    def _get(self, b: int) -> _Bucket:
        e = self._b.get(b)
        if e is not None:
            return e
        sizes = self._sizes(b)
        S_b = self._caps(b)[0]
        buf = torch.zeros(sum(sizes), dtype=torch.int32, device=self.device)
        e = _Bucket(size=b, sizes=sizes, S=S_b, buf=buf)
        buf.copy_(torch.from_numpy(self.pack_static(None, b)))
        e.dstep = views(buf, sizes + [S_b, 0])[0]
        self._body(e)                                   # eager warm-up (lazy allocations)
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=self._pool):
            e.tokens = self._body(e)
        self._pool = g.pool()
        e.graph = g
        self._b[b] = e
        return e

    def run(self, step: StepInputs) -> Optional[torch.Tensor]:
        """Replays the bucket's graph for ``step``; returns the device tensor
        of sampled tokens (first ``len(step.logit_rows)`` entries valid), or
        None when the step does not fit a bucket."""
        b = self.bucket_for(step)
        if b is None:
            return None
        host = self.pack_static(step, b)
        if host is None:
            return None
        e = self._get(b)
        self.stager.to_device(host, out=e.buf)
        e.graph.replay()
        self.replays += 1
        return e.tokens
