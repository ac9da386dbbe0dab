"""hipGraph capture of engine steps (SURVEY §2.6 "hipGraph bucket capture",
BASELINE config 5: continuous-batching decode, hipGraph).

A serving step (tens of concurrent requests, a decode / jump-forward span
each, a few hundred tokens) costs a few ms of weight streaming on the GPU but
~300 kernel launches (32 layers x 9 ops + sampling); issued one by one from
Python the launches, not the GPU, set the step time.  Steps with at most
``max(BUCKETS)`` tokens are therefore replayed from a captured hipGraph
(``torch.cuda.CUDAGraph`` is the HIP graph API on ROCm).  A graph is keyed by
(token bucket, sequence-capacity class, block-table width class, split-KV
factor, cascade on / off), captured at start-up (``warm``) or lazily on first
use, after one eager warm-up of the same static step.  Every step of
a key uses ONE fixed int32 layout (``pack_static``):

* tokens padded to the bucket size (padding writes no KV: slot -1), sequence
  arrays padded with empty dummy sequences (at most ``max_seqs`` real ones),
  attention work lists padded with work items of an empty sequence (the
  kernel's early exit), a block table of the class width (32, 128, 512, ...
  blocks: a long-context step does not make every short step ship a
  128k-position table), grammar-allowed sets padded to empty rows;
* prefix copy-on-write block pairs padded with (-1, -1) (the copy kernel skips
  them), copied inside the graph ahead of the forward - a step that attaches
  new requests to a shared prefix replays like any other;
* long-context low-batch steps keep their split-KV decode attention (K6): the
  split factor is part of the key and its fp32 partials live in the graph pool;
* the per-step H2D copy lands in the key's static device buffer, then the
  graph replays copies + forward + fused LM-head/grammar/sampling (K9) and
  leaves the tokens in a static output; the sampler's RNG counter (request
  uid, sample index) travels in the buffer and the seed is constant, so
  nothing in the graph changes per step;
* cascade (shared-prefix) attention replays too: the prefix pass is launched
  over the bucket's token capacity and reads [pre_tokens, pre_keys] from the
  buffer (pre_tokens 0 = no cascade this step, every item exits at once),
  the per-sequence first own key (kv_begin) and the prefix block ids travel
  in it as well.
"""
from __future__ import annotations

import dataclasses
import os
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import ops
from ..utils.tracing import span
from .batch import BLOCK_SIZE, HostStager, StepInputs, build_work, tokens_per_item, views

# token buckets: every 64 rows above 64 (the GEMM tile plan's M granularity,
# so padding a step to its bucket adds no MFMA tiles), finer below (the
# weight-streaming kernel's M classes); measured at 80 intents/s, power-of-two
# buckets padded a 300-token step to 512 and cost 12 % of p50
BUCKETS = (8, 16, 32, 48, 64) + tuple(range(128, 1025, 64))
# sequence-capacity classes: a step of 6 requests does not carry (and launch
# empty attention work items for) 128 dummy sequences
SEQ_CLASSES = (8, 32, 128, 512, 2048)
ALLOWED_PER_ROW = 64
MAX_COPIES = 64
MIN_WIDTH = 32                 # block-table width classes: 32, 128, 512, ... blocks (x4)


@dataclasses.dataclass
class _Bucket:
    key: Tuple[int, int, int, int, int]
    sizes: List[int]
    S: int
    buf: torch.Tensor
    graph: object = None
    tokens: Optional[torch.Tensor] = None
    dstep: object = None
    csrc: Optional[torch.Tensor] = None
    cdst: Optional[torch.Tensor] = None


def _nw1_cutoff(t1: int) -> int:
    # the same cutoff batch.build_work uses to route a sequence to 1-wave items
    return int(os.environ.get("MCP_ATTN_NW1_CUTOFF", str(t1 * 2)))


class GraphRunner:
    def __init__(self, model, kv, temperature: float, seed: int, buckets=BUCKETS,
                 max_seqs: int = 256, bcast=None, sample: bool = True):
        self.model, self.kv = model, kv
        self.bcast = bcast          # TP driver: StepBroadcaster (workers mirror every graph)
        self.sample = sample        # False on TP workers: forward only
        self.device = model.device
        self.group = model.cfg.group
        self.mblk = (model.cfg.max_pos + BLOCK_SIZE - 1) // BLOCK_SIZE
        self.temperature, self.seed = float(temperature), int(seed)
        self.buckets = tuple(sorted(buckets))
        self.max_seqs = int(max_seqs)
        self._b: Dict[Tuple[int, int, int, int, int], _Bucket] = {}
        self._pool = None
        self.stager = HostStager(self.device)
        self.replays = 0
        self.replay_host_s = 0.0     # host time inside CUDAGraph.replay()
        self.captures = 0
        self.capture_s = 0.0
        self.warmed = False     # warm() ran: split keys are no longer captured lazily

    # ---------------------------------------------------------------- layout
    def _seq_cap(self, b: int, sb: Optional[int]) -> int:
        return min(b, self.max_seqs if sb is None else sb)

    def _caps(self, b: int, sb: Optional[int] = None):
        # memoised: read on every step's host path (bucket_for, pack_static)
        memo = self.__dict__.setdefault("_caps_memo", {})
        r = memo.get((b, sb))
        if r is None:
            r = memo[(b, sb)] = self._caps_compute(b, sb)
        return r

    def _caps_compute(self, b: int, sb: Optional[int] = None):
        t1 = tokens_per_item(1, self.group)
        t4 = tokens_per_item(4, self.group)
        n = self._seq_cap(b, sb)
        S = n + 1                          # >= one empty dummy sequence
        cutoff = _nw1_cutoff(t1)
        cap1 = min(b, n * -(-cutoff // t1))              # 1-wave items: ql <= cutoff
        cap4 = min(b // t4 + n, b) + 1                   # 4-wave items: ceil(ql / t4)
        return S, cap1, cap4, S * ALLOWED_PER_ROW

    def _ncopy(self, b: int, sb: Optional[int] = None) -> int:
        return min(self._caps(b, sb)[0], MAX_COPIES)

    def _sizes(self, b: int, width: Optional[int] = None, sb: Optional[int] = None) -> List[int]:
        S, cap1, cap4, A = self._caps(b, sb)
        w = self.mblk if width is None else width
        C = self._ncopy(b, sb)
        # same part order as batch.pack_host / views
        return [b, b, b, S, S, S, S, S * w, cap1, cap1, cap4, cap4, C, C, S, 2 + w, S + 1, A, S]

    def width_for(self, need: int) -> Optional[int]:
        """Block-table width class for a step whose longest table has ``need``
        blocks (None past the model's context)."""
        if need > self.mblk:
            return None
        w = MIN_WIDTH
        while w < need:
            w *= 4
        return min(w, self.mblk)

    def seq_classes(self, b: int) -> List[int]:
        out = sorted({min(c, b, self.max_seqs) for c in SEQ_CLASSES})
        return out

    def bucket_for(self, step: StepInputs, ncopies: int = 0) -> Optional[Tuple[int, int]]:
        """(token bucket, sequence class) of the smallest static layout that
        holds ``step``, or None."""
        T = step.num_tokens
        S = int(step.q_len.shape[0])
        A = int(step.allow_ids.shape[0]) if step.allow_ids is not None else 0
        if step.block_table.shape[1] > self.mblk:
            return None
        for b in self.buckets:
            if T > b:
                continue
            for sb in self.seq_classes(b):
                Sb, _, _, Acap = self._caps(b, sb)
                if S < Sb and A <= Acap and ncopies <= self._ncopy(b, sb):
                    return b, sb
        return None

    def _template(self, b: int, w: int, sb: Optional[int]):
        """The packed static layout of (b, w, sb) at its defaults (padding
        rows, no slot, empty work lists pointing at the dummy sequence), made
        once; each step copies it and fills views of the copy (one memcpy
        instead of ~20 arrays and a concatenate on every step's host path)."""
        memo = self.__dict__.setdefault("_tmpl_memo", {})
        key = (b, w, sb)
        r = memo.get(key)
        if r is None:
            S_b, cap1, cap4, A_cap = self._caps(b, sb)
            sizes = self._sizes(b, w, sb)
            buf = np.zeros(sum(sizes), np.int32)
            offs = np.cumsum([0] + sizes)
            parts = [(int(offs[i]), int(offs[i + 1])) for i in range(len(sizes))]
            buf[parts[2][0]:parts[2][1]] = -1          # slots
            buf[parts[8][0]:parts[8][1]] = S_b - 1     # ws1
            buf[parts[10][0]:parts[10][1]] = S_b - 1   # ws4
            buf[parts[12][0]:parts[12][1]] = -1        # csrc
            buf[parts[13][0]:parts[13][1]] = -1        # cdst
            r = memo[key] = (buf, parts)
        return r

    def pack_static(self, step: Optional[StepInputs], b: int, width: Optional[int] = None,
                    copies: Sequence = (), sb: Optional[int] = None) -> Optional[np.ndarray]:
        S_b, cap1, cap4, A_cap = self._caps(b, sb)
        w = self.mblk if width is None else width
        C = self._ncopy(b, sb)
        T = step.num_tokens if step is not None else 0
        S = int(step.q_len.shape[0]) if step is not None else 0
        tmpl, parts = self._template(b, w, sb)
        out = tmpl.copy()
        (ids, pos, slots, rows, qs, ql, cl, bt, ws1, wq1, ws4, wq4, csrc, cdst, kvb, pre, aptr,
         aids, ctr) = (out[a:e] for a, e in parts)
        bt = bt.reshape(S_b, w)                    # pre: [pre_tokens, pre_keys, prefix blocks]
        if len(copies) > C:
            return None
        for i, (s_, d_) in enumerate(copies):
            csrc[i], cdst[i] = s_, d_
        if step is not None:
            if step.block_table.shape[1] > w:
                return None
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
            if step.pre_tokens > 0 and step.pre_bt is not None and len(step.pre_bt):
                nb = len(step.pre_bt)
                if nb > w:
                    return None
                kvb[:S] = step.kv_begin
                pre[0], pre[1] = step.pre_tokens, nb * BLOCK_SIZE
                pre[2:2 + nb] = step.pre_bt
            if R:
                aptr[:R + 1] = step.allow_ptr
                aptr[R + 1:] = step.allow_ptr[-1]
                A = int(step.allow_ids.shape[0])
                if A > A_cap:
                    return None
                aids[:A] = step.allow_ids
                ctr[:R] = step.sample_ctr
        return out

    # ---------------------------------------------------------------- graphs
    def _body(self, e: _Bucket):
        ops.copy_blocks(self.kv.data, e.csrc, e.cdst)
        hidden = self.model.forward(e.dstep, self.kv)
        if not self.sample:
            return None
        return ops.sample_allowed(hidden, self.model.w.lm_head, e.dstep.allow_ptr,
                                  e.dstep.allow_ids, e.dstep.sample_ctr, self.temperature,
                                  self.seed)

    def get(self, key) -> _Bucket:
        """The captured graph of ``key`` (capturing it on first use)."""
        return self._get(tuple(int(x) for x in key))

    def replay(self, key) -> None:
        """TP worker: replay ``key`` on the payload already in its buffer."""
        self._b[tuple(int(x) for x in key)].graph.replay()
        self.replays += 1

    def _get(self, key: Tuple[int, int, int, int, int]) -> _Bucket:
        e = self._b.get(key)
        if e is not None:
            return e
        t0 = time.perf_counter()
        b, sb, w, ns, casc = key
        sizes = self._sizes(b, w, sb)
        S_b = self._caps(b, sb)[0]
        buf = torch.zeros(sum(sizes), dtype=torch.int32, device=self.device)
        e = _Bucket(key=key, sizes=sizes, S=S_b, buf=buf)
        buf.copy_(torch.from_numpy(self.pack_static(None, b, w, sb=sb)))
        # pre_tokens -1: cascade sizes live on the device (batch.views); the
        # graphs of non-cascade steps launch no prefix pass at all
        e.dstep, e.csrc, e.cdst = views(buf, sizes + [S_b, -1 if casc else 0, ns, 1])
        self._body(e)                                   # eager warm-up (lazy allocations)
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        # thread_local: another host thread's work on its own stream (the
        # planner's prep thread running a retrieval search, MCP_PREP_THREAD)
        # may proceed while this thread captures a lazily built bucket
        mode = "thread_local" if os.environ.get("MCP_PREP_THREAD", "1") == "1" else "global"
        with torch.cuda.graph(g, pool=self._pool, capture_error_mode=mode):
            e.tokens = self._body(e)
        self._pool = g.pool()
        e.graph = g
        self._b[key] = e
        self.captures += 1
        self.capture_s += time.perf_counter() - t0
        return e

    # split-KV keys captured at start-up: the power-of-two split counts
    # (batch.choose_kv_splits) of few-sequence decode steps, in the buckets of
    # such steps; any other split key runs eagerly (no lazy capture on the
    # request path)
    WARM_SPLITS = (2, 4, 8)
    WARM_SPLIT_MAX_TOKENS = int(os.environ.get("MCP_WARM_SPLIT_MAX_TOKENS", "64"))
    WARM_SPLIT_SEQ_CLASSES = int(os.environ.get("MCP_WARM_SPLIT_SEQ_CLASSES", "1"))

    def warm(self, max_tokens: Optional[int] = None, contexts: Sequence[int] = (2048,),
             kv_splits: Sequence[int] = (1,)) -> int:
        """Capture every bucket up to ``max_tokens`` for the block-table width
        classes of ``contexts`` (tokens) ahead of serving, so no request waits
        on a lazy capture; plus the split-KV keys of small-batch decode
        (``WARM_SPLITS`` for the smallest sequence class of the buckets up to
        ``WARM_SPLIT_MAX_TOKENS``).  Returns the number of graphs captured."""
        n0 = self.captures
        widths = sorted({self.width_for((c + BLOCK_SIZE - 1) // BLOCK_SIZE) or self.mblk
                         for c in contexts})

        def cap(key, b, w, sb):
            if self.bcast is not None:                  # workers capture in lockstep
                self._launch_tp(key, self.pack_static(None, b, w, sb=sb))
            else:
                self._get(key)

        for b in self.buckets:
            if max_tokens is not None and b > max_tokens:
                break
            for sb in self.seq_classes(b):
                for w in widths:
                    for ns in kv_splits:
                        for casc in (0, 1):
                            cap((b, sb, w, int(ns), casc), b, w, sb)
            if b <= self.WARM_SPLIT_MAX_TOKENS and self.device.type == "cuda":
                for sb in self.seq_classes(b)[:self.WARM_SPLIT_SEQ_CLASSES]:
                    for w in widths:
                        for ns in self.WARM_SPLITS:
                            if ns in kv_splits:
                                continue
                            for casc in (0, 1):
                                cap((b, sb, w, int(ns), casc), b, w, sb)
        self.warmed = True
        return self.captures - n0

    def run(self, step: StepInputs, copies: Sequence = (), kv_splits: int = 1,
            pre=None) -> Optional[torch.Tensor]:
        """Replays the graph for ``step`` (after the prefix copy-on-write
        ``copies``); returns the device tensor of sampled tokens (first
        ``len(step.logit_rows)`` entries valid), or None when the step does
        not fit a bucket (the caller runs it eagerly).  ``pre(dstep)`` runs on
        the bucket's views between the payload copy and the replay (the
        engine's decision lookahead)."""
        bs = self.bucket_for(step, len(copies))
        if bs is None:
            return None
        b, sb = bs
        w = self.width_for(int(step.block_table.shape[1]))
        if w is None:
            return None
        with span("graph.pack"):
            host = self.pack_static(step, b, w, copies, sb)
        if host is None:
            return None
        casc = int(step.pre_tokens > 0 and step.pre_bt is not None and len(step.pre_bt) > 0)
        key = (b, sb, w, int(kv_splits), casc)
        if kv_splits > 1 and self.warmed and key not in self._b:
            return None        # an uncommon split key: eager, never a lazy capture mid-serving
        if self.bcast is not None:
            if pre is not None:
                return None
            e = self._launch_tp(key, host)
        else:
            e = self._get(key)
            with span("graph.h2d"):
                self.stager.to_device(host, out=e.buf)
            if pre is not None:
                pre(e.dstep)
            t0 = time.perf_counter()
            with span("graph.replay"):
                e.graph.replay()
            self.replay_host_s += time.perf_counter() - t0
        self.replays += 1
        return e.tokens

    def _launch_tp(self, key, host: np.ndarray) -> _Bucket:
        """TP driver: key to the workers (they capture it too if new, running
        the same eager warm-up collectives), then the payload into every
        rank's bucket buffer, then every rank replays."""
        self.bcast.send_graph(key, int(host.size))
        e = self._get(key)
        d = self.stager.to_device(host, out=e.buf)
        self.bcast.send_payload(d)
        e.graph.replay()
        return e
