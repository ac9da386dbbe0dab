"""Continuous-batching, grammar-driven LLM engine (one per GPU / TP group).

Replaces the remote LLM call of the reference planner (control_plane.py:69-73).
One ``step()`` = one ragged forward over every runnable sequence:

* a sequence contributes all its *pending* tokens: prompt chunks, the token
  sampled last step, and grammar-forced spans (jump-forward: forced JSON text
  is fed in the same forward instead of one decode step per token);
* KV goes into the paged cache; the shared registry-prompt prefix is computed
  once (per batch in the benchmark) by a prefix job; every request then shares
  its full blocks (reference counted) and gets a device-side copy of the
  partial tail block (copy-on-write) instead of recomputing those tokens;
* sequences waiting on a grammar choice get their last hidden state
  normalised and sampled by the fused allowed-set LM-head kernel (K9) at
  temperature 0.2 (control_plane.py:72);
* one host<->device round trip per step: packed int32 metadata in, sampled
  token ids out.

The scheduler is single-threaded and owns all GPU state; the
async frontend (planner.local) talks to it through queues.
"""
from __future__ import annotations

import dataclasses
import os
import itertools
import time
from typing import Callable, Dict, List, Optional, Sequence as Seq

import numpy as np
import torch

from .. import ops
from ..utils.metrics import METRICS
from ..utils.tracing import span
from .batch import BLOCK_SIZE, HostStager, choose_kv_splits, pack_step, step_from_host, views
from .kv_cache import KVCache

# steps above this many tokens run eagerly even when a graph bucket fits.  At
# serving loads the bigger steps (tens of requests) ran slower replayed than
# eager - the padded token bucket, work lists and block table of the graph key
# cost more than the launches they save: config 5 at 120 intents/s p50 328 ->
# 304 ms, 20/s 124 -> 122, 80/s 188 -> 187, config 2 96.4 -> 95.8 with 128
# (profiles/graph_max_tokens_ab.jsonl).  MCP_GRAPH_MAX_TOKENS overrides
_GRAPH_MAX_T = int(os.environ.get("MCP_GRAPH_MAX_TOKENS", "128"))

_uid = itertools.count(1)


@dataclasses.dataclass
class PrefixEntry:
    tokens: tuple
    blocks: List[int]          # ceil(length / 64) blocks; the last may be partial
    length: int                # prefix tokens
    computed: bool = False
    hashes: tuple = ()         # chained hashes of the full 64-token blocks
    shared: int = 0            # leading blocks taken from other cached prefixes


def block_hashes(tokens: Seq[int]) -> tuple:
    """Chained hash of every full 64-token block: block i's hash covers
    tokens [0, 64 (i + 1)), so equal hashes mean equal KV for that block."""
    out, h = [], 0
    for b in range(len(tokens) // BLOCK_SIZE):
        h = hash((h, tuple(tokens[b * BLOCK_SIZE:(b + 1) * BLOCK_SIZE])))
        out.append(h)
    return tuple(out)


class Sequence:
    def __init__(self, decoder, prompt_tokens: List[int], prefix: Optional[PrefixEntry] = None,
                 on_done: Optional[Callable] = None):
        self.uid = next(_uid)
        self.decoder = decoder
        self.prefix = prefix
        self.materialized = prefix is None
        self.blocks: List[int] = []
        self.num_cached = 0                    # tokens whose KV is in this sequence's blocks
        self.pending: List[int] = list(prompt_tokens)
        # every token of the request after its shared prefix (prompt + grammar
        # output); ``pending`` is always a suffix of it - a preempted request
        # recomputes prefix + tokens
        self.tokens: List[int] = list(prompt_tokens)
        self.base = 0                          # leading tokens (shared prefix) not in `tokens`
        self.evicted = False                   # preempted during the current schedule
        self.n_samples = 0
        self.done = False
        self.result = None
        self.error: Optional[str] = None
        self.on_done = on_done
        self.t_submit = time.perf_counter()
        self.t_admit = None
        self.t_first = None
        self.t_done = None
        self.is_prefix_job = decoder is None
        self.cohort = 0                        # launch cohort (pipelined engine)
        if decoder is not None:
            first = decoder.advance()
            self.pending += first
            self.tokens += first

    @property
    def wants_sample(self) -> bool:
        return self.decoder is not None and not self.decoder.done


@dataclasses.dataclass
class _Launch:
    """One forward in flight: what to update once its sampled tokens land."""
    batch_seqs: list
    sample_seqs: list
    tokens: Optional[torch.Tensor]      # host (pinned) copy of the sampled tokens
    event: Optional[object]             # completion of the D2H copy
    T: int
    booked: bool = False                # batch_seqs' launched tokens already counted
    tok_dev: Optional[torch.Tensor] = None   # device sampled tokens (row i = sample i)
    # decision lookahead (_launch_branch): the sequences in sample-row order and,
    # per sequence, token -> (token, appended tokens, done, next allowed, decoder)
    seqs: Optional[list] = None
    branches: Optional[list] = None


# MCP_SPIN_WAIT=1: busy-poll the sampled-token event (one host core per GPU
# process spins during the forward) instead of blocking in hipEventSynchronize.
# Measured no faster (headline 216.6 / 215.6 vs 216.6 / 217.1 plans/s, 40
# intents/s p50 171.1 vs 170.6 ms, same box): off by default
_SPIN_WAIT = os.environ.get("MCP_SPIN_WAIT", "0") == "1"

# MCP_LOOKAHEAD=1: decision lookahead for small batches (single intent /
# low-QPS serving).  The next forward is launched before the host has read
# this step's sampled tokens: laid out for every outcome of each sequence's
# pending grammar choice (native decoder clones give each outcome's forced
# span and next allowed set), the device picks the sampled outcome
# (csrc/sampling.hip branch_select_kernel) between the step's H2D copy and its
# forward.  The host's per-decision work (read-back, grammar, schedule, pack,
# launch) then runs while the GPU is busy with the next step instead of
# between steps.
# On by default since round 6: with the hold (LLMEngine.LOOK_HOLD) an arrival
# joins the branch step instead of queueing behind it; same box, alternated
# (profiles/lookahead_hold_ab_r6.txt): config 2 p50 85.2-85.4 vs 85.8-86.9 ms,
# config 5 at 20 / 40 intents/s p50 103.1-103.4 / 115.3-115.7 vs 103.7-105.0 /
# 121.6-121.9 ms, at 80/s 144.3 vs 142.8 (one round).  MCP_LOOKAHEAD=0: off.
_LOOKAHEAD = os.environ.get("MCP_LOOKAHEAD", "1") == "1"


def tp_graph_safe(model) -> bool:
    """TP: workers mirror the driver's graphs, so every collective a bucket
    runs must be capturable - the all-reduces (K12 / RCCL, not gloo on GPU
    tensors) and, with sequence parallelism, the reduce-scatter / all-gather
    pair (``parallel.comm.make_sp_collectives`` tags them)."""
    from .graphs import BUCKETS
    safe = getattr(getattr(model, "_allreduce", None), "graph_safe", None)
    if safe is None or not safe(max(BUCKETS) * model.cfg.hidden * 2):
        return False
    if getattr(model, "seq_parallel", False):
        return all(getattr(f, "graph_safe", False) for f in (model._sp or ()))
    return True


_FEED_ADVANCE = False


def _native_feed_advance():
    """(runtime.feed_advance_many, native DagDecoder type, runtime.allowed_many) or None."""
    global _FEED_ADVANCE
    if _FEED_ADVANCE is False:
        _FEED_ADVANCE = None
        from . import native
        rt = native._RT if native.available() else None
        if rt is not None and hasattr(rt, "allowed_many") and hasattr(rt, "DagDecoder"):
            _FEED_ADVANCE = (rt.feed_advance_many, rt.DagDecoder, rt.allowed_many)
    return _FEED_ADVANCE


class LLMEngine:
    def __init__(self, model, num_blocks: Optional[int] = None, kv_budget_bytes: Optional[int] = None,
                 max_batch: int = 256, max_step_tokens: int = 8192, temperature: float = 0.2,
                 seed: int = 0, bcast=None, cascade: bool = True, pipeline: Optional[bool] = None,
                 graphs: Optional[bool] = None, lookahead: Optional[bool] = None):
        self.model = model
        cfg = model.cfg
        self.device = model.device
        self.bcast = bcast          # parallel.comm.StepBroadcaster on a TP driver, else None
        self.cascade = cascade and os.environ.get("MCP_CASCADE", "1") == "1"   # shared-prefix attention
        # optional two launch cohorts in flight: the host schedules / updates one
        # cohort while the GPU runs the other's forward.  Every cohort step
        # streams all the weights again, so a request waits two weight-bound
        # steps per sampled token: measured on one MI355X (config 5, same run)
        # p50 368 / 464 / 594 ms with cohorts vs 194 / 242 / 572 ms without at
        # 40 / 80 / 160 intents/s (profiles/config5_pipeline_ab.jsonl).  Off by
        # default; "auto" = cohorts only while >= PIPELINE_MIN_SEQS requests run
        # (160 / 200 intents/s: 615 / 1170 ms, no better than off).
        if pipeline is None:
            env = os.environ.get("MCP_PIPELINE", "0")
            pipeline = "auto" if env == "auto" else env == "1"
        if pipeline == "auto" and self.device.type != "cuda":
            pipeline = False
        self.pipeline = pipeline
        self.inflight: Dict[int, _Launch] = {}
        self.lookahead = (_LOOKAHEAD if lookahead is None else bool(lookahead)) and bcast is None
        self._look: List[_Launch] = []          # [launch whose samples decide, branch launch]
        self._look_err = None
        # lookahead hold (_look_hold): the driver's arrival pump, and the
        # measured device time of one lookahead step
        self.poll_arrivals: Optional[Callable[[], int]] = None
        self._look_step_s = 0.0
        self._look_ready_t = None
        self.last_progress = time.perf_counter()   # watched by the planner's stall watchdog
        self._turn = 0
        self._next_cohort = 0
        self.stager = HostStager(self.device)
        self._look_stager = HostStager(self.device)
        if graphs is None:
            graphs = self.device.type == "cuda" and os.environ.get("MCP_GRAPHS", "1") == "1"
            if graphs and getattr(model, "tp", 1) > 1:
                graphs = bcast is not None and tp_graph_safe(model)
        self._graphs_wanted = graphs
        self.graphs = None          # engine.graphs.GraphRunner, created after the KV cache
        if num_blocks is not None:
            self.kv = KVCache(cfg.layers, model.hkv, cfg.head_dim, num_blocks, self.device)
        else:
            self.kv = KVCache.sized_for(cfg.layers, model.hkv, cfg.head_dim, self.device,
                                        budget_bytes=kv_budget_bytes)
        self.alloc = self.kv.allocator
        self.max_batch = max_batch
        self.max_step_tokens = max_step_tokens
        # chunked prefill (MCP_PREFILL_CHUNK tokens per step, 0 = off): while
        # any request is past its first sample (decoding: one decision + its
        # forced span per step), requests still in their prompt take at most
        # this many prompt tokens per step between them, so a long
        # (retrieval-sized) prompt no longer stretches every running
        # request's decision step to a whole-prompt forward (config 3)
        self.prefill_chunk = int(os.environ.get("MCP_PREFILL_CHUNK", "0"))
        # decode priority: with MCP_PREFILL_DECODE_REF = r
        # > 0 the prompt budget shrinks as decoding requests grow - the chunk
        # while at most r requests decode, chunk * r / n with n decoding,
        # never below MCP_PREFILL_MIN - so a step's decisions stay cheap when
        # many requests wait on them, and prompts go faster when few do
        self.prefill_decode_ref = int(os.environ.get("MCP_PREFILL_DECODE_REF", "0"))
        self.prefill_min = int(os.environ.get("MCP_PREFILL_MIN", "64"))
        self.temperature = temperature
        self.seed = seed
        self.running: List[Sequence] = []
        self.waiting: List[Sequence] = []
        self._deferred_free: List[int] = []              # released after the step's copies are queued
        self.prefixes: Dict[tuple, PrefixEntry] = {}     # insertion order = LRU order
        self._last_prefix = None                         # (token list object, entry)
        self.max_prefixes = 64
        # block-level prefix reuse: chained block hash -> keys of cached
        # entries holding that block (a new prefix shares the leading full
        # blocks it has in common with any computed entry, e.g. retrieved
        # service lists that start with the same services; MCP_BLOCK_REUSE=0
        # disables)
        self._block_index: Dict[int, Dict[tuple, int]] = {}
        self.block_reuse = os.environ.get("MCP_BLOCK_REUSE", "1") == "1"
        self.steps = 0
        if self._graphs_wanted:
            from .graphs import GraphRunner
            self.graphs = GraphRunner(model, self.kv, temperature, seed, max_seqs=max_batch,
                                      bcast=bcast)
        self.stats = {"tokens": 0, "samples": 0, "steps": 0, "graph_steps": 0, "graph_cow_steps": 0,
                      "graph_split_steps": 0, "graph_cascade_steps": 0, "kv_split_steps": 0, "preemptions": 0,
                      "schedule_s": 0.0, "launch_s": 0.0, "sample_s": 0.0, "update_s": 0.0,
                      "lookahead_steps": 0, "lookahead_admitted": 0}

    # ------------------------------------------------------------- prefixes
    def get_prefix(self, tokens: Seq[int]) -> Optional[PrefixEntry]:
        """Shared prefix entry for ``tokens``; the first request creates a
        prefix job that computes the prefix KV once."""
        # the planner hands every request of a batch the same cached token list:
        # skip re-tupling / re-hashing ~700 tokens per request
        last = self._last_prefix
        if last is not None and last[0] is tokens and self.prefixes.get(last[1].tokens) is last[1]:
            return last[1]
        src = tokens
        tokens = tuple(tokens)
        if len(tokens) < BLOCK_SIZE:
            return None
        e = self.prefixes.pop(tokens, None)
        if e is not None:
            self.prefixes[tokens] = e                  # refresh LRU position
        else:
            while len(self.prefixes) >= self.max_prefixes:   # evict the LRU entry
                self._drop_entry(next(iter(self.prefixes)))
            need = (len(tokens) + BLOCK_SIZE - 1) // BLOCK_SIZE
            hashes = block_hashes(tokens) if self.block_reuse else ()
            shared = self._shared_blocks(tokens, hashes)
            self.alloc.incref(shared)          # held before eviction can drop their entries
            # a full pool: drop cached prefixes before giving up sharing -
            # with retrieval every request may bring its own prefix
            if not self._evict_prefixes(need - len(shared)):
                if shared:
                    self.alloc.free(shared)
                return None             # the request carries its whole prompt instead
            blocks = shared + self.alloc.alloc(need - len(shared))
            e = PrefixEntry(tokens=tokens, blocks=blocks, length=len(tokens), hashes=hashes,
                            shared=len(shared))
            self.prefixes[tokens] = e
            for i, h in enumerate(hashes):
                self._block_index.setdefault(h, {})[tokens] = i
            n_sh = len(shared) * BLOCK_SIZE
            job = Sequence(None, list(tokens[n_sh:]))
            job.blocks = list(blocks)
            job.num_cached = n_sh               # the shared blocks' keys are computed
            job.prefix_entry = e
            self.alloc.incref(blocks)          # the job's own reference
            self.waiting.insert(0, job)
            self.stats["prefix_blocks"] = self.stats.get("prefix_blocks", 0) + need
            self.stats["prefix_blocks_reused"] = self.stats.get("prefix_blocks_reused", 0) + len(shared)
        self._last_prefix = (src, e)
        return e

    def _shared_blocks(self, tokens: tuple, hashes: tuple) -> List[int]:
        """The leading full blocks of ``tokens`` that computed cached entries
        already hold (longest run of matching chained hashes, tokens checked)."""
        out = []
        for i, h in enumerate(hashes):
            holders = self._block_index.get(h)
            src = None
            for key in holders or ():
                ent = self.prefixes.get(key)
                if ent is not None and ent.computed and ent.tokens[:(i + 1) * BLOCK_SIZE] == \
                        tokens[:(i + 1) * BLOCK_SIZE]:
                    src = ent
                    break
            if src is None:
                break
            out.append(src.blocks[i])
        # keep at least one token to compute: the prefix job must run a step
        if out and len(out) * BLOCK_SIZE >= len(tokens):
            out.pop()
        return out

    def _drop_entry(self, key: tuple) -> None:
        """Forget one cached prefix: release its blocks (requests and other
        entries sharing them keep theirs) and its block-index entries."""
        e = self.prefixes.pop(key)
        for h in e.hashes:
            holders = self._block_index.get(h)
            if holders is not None:
                holders.pop(key, None)
                if not holders:
                    del self._block_index[h]
        if self._last_prefix is not None and self._last_prefix[1] is e:
            self._last_prefix = None
        self.alloc.free(e.blocks)

    def _evict_prefixes(self, need: int) -> bool:
        """Drop cached prefix entries, least recently used first, until
        ``need`` blocks are free.  Entries no request uses go first (every
        block returns to the pool); then entries that free at least one block
        (a prefix whose full blocks running requests still share gives back
        its tail); an entry whose blocks are all still shared frees nothing
        and stays cached - dropping it would only make later requests
        recompute a hot prefix.  Returns whether ``need`` blocks are free."""
        a = self.alloc
        if a.num_free >= need:
            return True
        for only_unused in (True, False):
            for key in list(self.prefixes):
                if a.num_free >= need:
                    return True
                blocks = self.prefixes[key].blocks
                held = sum(1 for b in blocks if a.refcount(b) == 1)
                if held == 0 or (only_unused and held < len(blocks)):
                    continue
                self._drop_entry(key)
        return a.num_free >= need

    def _alloc_pressure(self, need: int, protect: set) -> Optional[List[int]]:
        """``need`` blocks when the pool is short: evict cached prefixes, then
        preempt running requests (most recently admitted first) that are
        neither in ``protect`` (this step's batch) nor in a launch still in
        flight.  None when even that does not free enough."""
        if not self._evict_prefixes(need):
            busy = set(protect)
            for L in self.inflight.values():
                busy.update(id(q) for q, _ in L.batch_seqs)
            for seq in list(reversed(self.running)):    # _preempt edits running
                if self.alloc.num_free >= need:
                    break
                if seq.is_prefix_job or seq.evicted or not seq.blocks or id(seq) in busy:
                    continue
                self._preempt(seq)
            if self.alloc.num_free < need:
                return None
        return self.alloc.alloc(need)

    def _preempt(self, seq: Sequence):
        """Preemption by recompute: keep the shared full blocks of the
        request's prefix, free the rest and queue it at the front of
        ``waiting`` with everything after them (the prefix's partial tail
        block + its own tokens) pending again; its grammar state and sample
        counter carry on."""
        keep = seq.base // BLOCK_SIZE
        head = list(seq.prefix.tokens[keep * BLOCK_SIZE:seq.base]) if seq.base % BLOCK_SIZE else []
        if keep and seq.prefix is not None:
            seq.kept_prefix = seq.prefix       # its first ``keep`` blocks stay shared
        self.alloc.free(seq.blocks[keep:])
        del seq.blocks[keep:]
        seq.pending = head + seq.tokens
        seq.tokens = list(seq.pending)
        seq.base = seq.num_cached = keep * BLOCK_SIZE
        seq.prefix = None                      # no cascade for it: its keys are its own
        seq.evicted = True
        self.running.remove(seq)
        self.waiting.insert(0, seq)
        self.stats["preemptions"] += 1

    def _release_idle(self, need: int, skip) -> None:
        """Last resort before failing a request for memory: requests that are
        not in this step hold shared-prefix blocks too - preempted ones keep
        their prefix's full blocks, not-yet-materialised ones a reference to
        their whole prefix.  Fully release them (most recently queued first)
        until ``need`` blocks are free; each then carries its whole prompt as
        pending tokens."""
        a = self.alloc
        for seq in list(reversed(self.waiting)) + list(reversed(self.running)):
            if a.num_free >= need:
                return
            if seq is skip or seq.is_prefix_job or seq.done:
                continue
            if not seq.materialized:
                e = seq.prefix
                a.free(e.blocks)
                seq.pending = list(e.tokens) + seq.pending
                seq.tokens = list(e.tokens) + seq.tokens
                seq.prefix, seq.materialized = None, True
            elif seq.evicted or seq in self.waiting:
                if not seq.blocks:
                    continue
                kept = getattr(seq, "kept_prefix", None)
                if kept is None or seq.num_cached != seq.base:
                    continue                   # holds KV of its own: not a prefix-only holder
                a.free(seq.blocks)
                seq.blocks = []
                head = list(kept.tokens[:seq.base])
                seq.pending = head + seq.pending
                seq.tokens = head + seq.tokens
                seq.base = seq.num_cached = 0
                seq.kept_prefix = None
            else:
                continue
            self.stats["released"] = self.stats.get("released", 0) + 1

    def _blocks_to_admit(self, seq: Sequence) -> int:
        """Blocks a waiting request needs for the tokens it already has."""
        if seq.materialized:
            return (seq.num_cached + len(seq.pending) + BLOCK_SIZE - 1) // BLOCK_SIZE - len(seq.blocks)
        e = seq.prefix                         # shares e's full blocks, copies the tail
        return (e.length + len(seq.pending) + BLOCK_SIZE - 1) // BLOCK_SIZE - e.length // BLOCK_SIZE

    def drop_prefixes(self):
        """Release prefix entries (their blocks stay alive while requests use them)."""
        for e in self.prefixes.values():
            self.alloc.free(e.blocks)
        self.prefixes.clear()
        self._block_index.clear()
        self._last_prefix = None

    def _materialize(self, seq: Sequence, copies: list):
        """Attach a request to its computed prefix: share the full blocks, copy
        the partial tail block (device copy queued before the next forward)."""
        e = seq.prefix
        n_full, tail = divmod(e.length, BLOCK_SIZE)
        nb = None
        if tail:
            got = self.alloc.alloc(1) if self.alloc.num_free else self._alloc_pressure(1, set())
            if got is None:
                return False                   # pool exhausted: retry on a later step
            nb = got[0]
        seq.blocks = list(e.blocks[:n_full])
        if tail:
            copies.append((e.blocks[-1], nb))
            seq.blocks.append(nb)
            # the reference taken at submit is released only after this
            # step's copies are queued: freed now (an already evicted prefix
            # drops the block's last reference), the LIFO pool could hand the
            # block to another request's tail copy in the same step - copy
            # pairs (t_a -> n_a), (t_b -> t_a) run in parallel and a's tail
            # would take b's KV
            self._deferred_free.append(e.blocks[-1])
        seq.num_cached = seq.base = e.length
        seq.materialized = True
        return True

    # ------------------------------------------------------------ requests
    def submit(self, decoder, prompt_tokens: List[int], prefix_tokens: Optional[List[int]] = None,
               on_done: Optional[Callable] = None) -> Sequence:
        """Queue one grammar-constrained generation.  ``prefix_tokens`` is the
        shareable leading part of the prompt (registry section)."""
        total = len(prefix_tokens or ()) + len(prompt_tokens)
        max_pos = getattr(self.model.cfg, "max_pos", None)
        if max_pos is not None and total >= max_pos:
            raise ValueError(f"prompt of {total} tokens does not fit the model's "
                             f"{max_pos}-token context")
        prefix = self.get_prefix(prefix_tokens) if prefix_tokens else None
        if prefix is not None:
            self.alloc.incref(prefix.blocks)
            seq = Sequence(decoder, list(prompt_tokens), prefix, on_done)
        else:
            seq = Sequence(decoder, list(prefix_tokens or []) + list(prompt_tokens), None, on_done)
        seq.cohort = self._next_cohort
        self._next_cohort ^= 1
        if not self.has_work():
            self.last_progress = time.perf_counter()
        self.waiting.append(seq)
        return seq

    def abort_all(self, reason: str = "aborted") -> int:
        """Fail every queued and running request (their blocks go back to the
        allocator) and forget the prefix cache: the planner's recovery after a
        stalled step.  Launches still in flight are waited for first.  Returns
        the number of requests failed."""
        for L in list(self.inflight.values()) + self._look:
            if L.event is not None:
                L.event.synchronize()
        self.inflight.clear()
        self._look = []
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        n = 0
        now = time.perf_counter()
        for seq in self.running + self.waiting:
            if seq.done:
                continue
            if seq.materialized or seq.is_prefix_job:
                self.alloc.free(seq.blocks)
            else:                                   # still holds its prefix reference
                self.alloc.free(seq.prefix.blocks)
            seq.blocks = []
            seq.done, seq.t_done = True, now
            if seq.is_prefix_job:
                continue
            seq.error = reason
            n += 1
            if seq.on_done is not None:
                seq.on_done(seq)
        self.running, self.waiting = [], []
        self.drop_prefixes()
        self.last_progress = time.perf_counter()
        return n

    def launch_ahead(self) -> bool:
        """Launch the next step now and retire it in the next ``step()``: a
        caller that is about to prepare more requests (suffix tokenisation of a
        batch) lets the GPU run the queued work - the batch's shared-prefix job
        - meanwhile.  Only on an idle engine (nothing running or in flight) and
        without the two-cohort pipeline; returns whether a step was launched.
        Headline A/B (same box, interleaved): 217.3 / 215.6 plans/s with it,
        215.4 / 219.1 without - within run-to-run noise (the overlap is the
        ~10 ms suffix tokenisation of a 256-intent batch)."""
        if self.pipeline or self.inflight or self._look or self.running or not self.waiting:
            return False
        L = self._schedule_launch(None)
        if L is None:
            return False
        self.inflight[-1] = L
        return True

    def has_work(self) -> bool:
        return bool(self.running or self.waiting or self.inflight or self._look)

    # ---------------------------------------------------------------- step
    def _admit(self):
        """FIFO admission while the batch has room and the pool holds the
        blocks of the admitted requests' current tokens (an empty batch admits
        regardless; a request the whole pool cannot hold fails at schedule)."""
        free = None
        while self.waiting and len(self.running) < self.max_batch:
            seq = self.waiting[0]
            if not seq.is_prefix_job:
                need = self._blocks_to_admit(seq)
                if free is None:
                    free = self.alloc.num_free
                if need > free:
                    before = self.alloc.num_free
                    self._evict_prefixes(before + need - free)
                    free += self.alloc.num_free - before
                    if need > free and self.running:
                        break
                free -= need
            self.waiting.pop(0)
            seq.evicted = False
            if seq.t_admit is None:
                seq.t_admit = time.perf_counter()
            self.running.append(seq)

    def _ensure_blocks(self, seq: Sequence, total_tokens: int):
        need = (total_tokens + BLOCK_SIZE - 1) // BLOCK_SIZE - len(seq.blocks)
        if need > 0:
            seq.blocks += self.alloc.alloc(need)

    def _finish(self, seq: Sequence):
        seq.done = True
        seq.t_done = time.perf_counter()
        self.alloc.free(seq.blocks)
        seq.blocks = []
        if seq.is_prefix_job:
            seq.prefix_entry.computed = True
        else:
            t_parse = time.perf_counter()
            if seq.error is None:
                try:
                    seq.result = seq.decoder.result()
                except Exception as e:  # pragma: no cover - grammar guarantees JSON
                    seq.error = repr(e)
            METRICS.observe("parse_s", time.perf_counter() - t_parse)
            METRICS.plan_done(seq.t_done - seq.t_submit)
            # per-request phases: queue (submit -> admitted), first sampled
            # token (prefill), first token -> done (decode + jump-forward), total
            if seq.t_admit is not None:
                METRICS.observe("queue_s", seq.t_admit - seq.t_submit)
            if seq.t_first is not None:
                METRICS.observe("ttft_s", seq.t_first - seq.t_submit)
                METRICS.observe("decode_s", seq.t_done - seq.t_first)
            METRICS.inc("sampled_tokens", seq.n_samples)
        if seq.on_done is not None:
            seq.on_done(seq)

    def step(self) -> int:
        """Advance the engine by one launch.  Returns the tokens launched plus
        the tokens retired (0 = no progress).

        Pipelined: cohort c's previous launch is retired (its sampled tokens
        fed to the grammar) while the GPU is still busy with cohort c^1's
        forward, then cohort c is scheduled and launched asynchronously."""
        if self._look:
            return self._step_look()
        if not self._pipelined_now() or self._big_step():
            while self.inflight:                  # drain the cohorts before a full-batch step
                c, L = self.inflight.popitem()
                self._retire(L)
            with span("engine.launch"):
                L = self._schedule_launch(None)
            if L is None:
                return 0
            if self.lookahead and self._look_start(L):
                self.last_progress = time.perf_counter()
                return L.T
            with span("engine.retire"):
                self._retire(L)
            self.last_progress = time.perf_counter()
            return L.T
        c = self._turn
        self._turn ^= 1
        done = 0
        L = self.inflight.pop(c, None)
        if L is not None:
            with span("engine.retire"):
                self._retire(L)
            done = L.T
            self.last_progress = time.perf_counter()
        with span("engine.launch"):
            nxt = self._schedule_launch(c)
        if nxt is not None:
            self.inflight[c] = nxt
            return done + nxt.T
        return done

    PIPELINE_MAX_TOKENS = 1024
    CASCADE_MIN_SHARERS = 4
    PIPELINE_MIN_SEQS = 64

    def _pipelined_now(self) -> bool:
        if self.pipeline == "auto":
            return len(self.running) + len(self.waiting) >= self.PIPELINE_MIN_SEQS
        return bool(self.pipeline)

    def _big_step(self) -> bool:
        """Large batches run as ONE launch: halving the GEMM M per cohort costs
        more in MFMA wave quantisation (e.g. 112 tiles on 256 CUs) than the
        host time the two-cohort overlap hides (measured: 166 vs 156 plans/s at
        256 concurrent intents)."""
        n = 0
        for q in self.running:
            n += len(q.pending)
            if n > self.PIPELINE_MAX_TOKENS:
                return True
        return False

    def prefill_budget(self, n_decoding: int) -> int:
        """Prompt tokens one step may take while ``n_decoding`` requests are
        past their first sample (chunked prefill, decode priority)."""
        c, r = self.prefill_chunk, self.prefill_decode_ref
        if r <= 0 or n_decoding <= r:
            return c
        return max(min(c, self.prefill_min), c * r // n_decoding)

    def _schedule_launch(self, cohort: Optional[int]) -> Optional[_Launch]:
        try:
            return self._schedule_launch_inner(cohort)
        finally:
            if self._deferred_free:            # this step's copy list is queued on the stream
                self.alloc.free(self._deferred_free)
                self._deferred_free = []

    def _schedule_launch_inner(self, cohort: Optional[int]) -> Optional[_Launch]:
        t_sched = time.perf_counter()
        self._admit()
        if not self.running:
            return None
        pool = self.running if cohort is None else [q for q in self.running if q.cohort == cohort]
        copies = []
        unplaced = None                       # a computed-prefix request the pool could not take
        for seq in pool:
            if not seq.materialized and seq.prefix.computed:
                if not self._materialize(seq, copies):
                    unplaced = unplaced or seq
        if any(q.evicted for q in pool):     # preempted while materialising
            pool = [q for q in pool if not q.evicted]
        budget = self.max_step_tokens
        entries, sample_seqs, batch_seqs = [], [], []
        T = 0
        # cascade: requests that share the most common computed prefix go first,
        # so their tokens form the leading range [0, pre_tokens) of the batch
        casc = None
        if self.cascade:
            counts = {}
            for seq in pool:
                e = seq.prefix
                if e is not None and seq.materialized and seq.pending and e.length >= BLOCK_SIZE:
                    counts[id(e)] = counts.get(id(e), 0) + 1
            if counts:
                best = max(counts, key=counts.get)
                n_share = counts[best]
                casc = next(q.prefix for q in pool if q.prefix is not None and id(q.prefix) == best)
                # the prefix pass has ~(sharing tokens / 32) x Hkv workgroups: for a
                # long prefix shared by few sequences that underfills the chip,
                # while per-sequence attention can split the key range (split-KV);
                # with a handful of sharers the per-sequence split-KV path is
                # faster at any prefix length (config 2, one intent: p50 121 ->
                # 113 ms, profiles/config2_attention_ab.jsonl)
                if (casc.length >= 16 * BLOCK_SIZE and n_share < 16) or n_share < self.CASCADE_MIN_SHARERS:
                    casc = None
        order = list(pool)                     # _alloc_pressure may preempt (edit running)
        if casc is not None:
            first, rest = [], []
            for q in pool:
                (first if (q.prefix is casc and q.materialized) else rest).append(q)
            order = first + rest
        pre_tokens = 0
        casc_keys = (casc.length // BLOCK_SIZE) * BLOCK_SIZE if casc is not None else 0
        alloc, pool_free = self.alloc.alloc, self.alloc
        blocked = None
        # chunked prefill: the prompt-token budget of this step, when decoding
        # requests share it (None: no cap)
        pf_left = None
        if self.prefill_chunk > 0:
            n_dec = sum(1 for q in order if q.n_samples > 0)
            if n_dec:
                pf_left = self.prefill_budget(n_dec)
        add_entry, add_batch, add_sample = entries.append, batch_seqs.append, sample_seqs.append
        # the per-request loop of every step (host critical path): locals bound,
        # _ensure_blocks / wants_sample inlined
        for seq in order:
            if not seq.materialized or seq.evicted:   # waiting for its prefix job / preempted
                continue
            pend = seq.pending
            n = len(pend)
            if n == 0:
                continue
            take = budget - T
            if take <= 0:
                break
            if n < take:
                take = n
            if pf_left is not None and seq.n_samples == 0 and seq.decoder is not None:
                if pf_left <= 0:
                    continue                   # its prompt goes on next step
                if take > pf_left:
                    take = pf_left
                pf_left -= take
            start = seq.num_cached
            blocks = seq.blocks
            need = (start + take + BLOCK_SIZE - 1) // BLOCK_SIZE - len(blocks)
            if need > 0:
                if need <= pool_free.num_free:
                    blocks += alloc(need)
                else:                          # memory pressure (rare): evict / preempt
                    got = self._alloc_pressure(need, {id(q) for q, _ in batch_seqs} | {id(seq)})
                    if got is None:
                        blocked = blocked or seq
                        continue
                    blocks += got
            T += take
            if casc is not None and seq.prefix is casc:
                pre_tokens = T
                ck = casc_keys
            else:
                ck = 0
            dec = seq.decoder
            sample = take == n and dec is not None and not dec.done
            add_entry((pend, take, start, blocks, ck, sample))
            add_batch((seq, take))
            if sample:
                add_sample(seq)
        group = self.model.cfg.group
        if T == 0:
            if copies:     # copy-on-write blocks still have to land before later steps
                self._launch(*pack_step([], BLOCK_SIZE, group, copies))
            if unplaced is not None and blocked is None and not self.inflight:
                # its tail block is held by idle requests' prefixes: release them
                self._release_idle(1, unplaced)
                self._evict_prefixes(1)
            if blocked is not None and not self.inflight:
                own = (blocked.num_cached + len(blocked.pending) + BLOCK_SIZE - 1) // BLOCK_SIZE
                if own > self.kv.num_blocks:
                    # the request alone does not fit the whole pool
                    blocked.error = (f"KV cache exhausted: the request needs {own} blocks, "
                                     f"the pool has {self.kv.num_blocks}")
                    self._finish(blocked)
                    self.running = [q for q in self.running if not q.done]
                else:
                    # it fits once the blocks idle requests hold are released
                    # (the next step schedules it)
                    want = own - len(blocked.blocks)
                    self._release_idle(want, blocked)
                    if not self._evict_prefixes(want):
                        blocked.error = (f"KV cache exhausted: the request needs {own} blocks, "
                                         f"{self.alloc.num_free} of {self.kv.num_blocks} can be freed")
                        self._finish(blocked)
                        self.running = [q for q in self.running if not q.done]
            return None
        allowed = ctr = None
        if sample_seqs:            # grammar masks go in the same single H2D copy
            with span("sched.allowed"):
                decs = [q.decoder for q in sample_seqs]
                fa = _native_feed_advance()
                if fa is not None and all(type(d) is fa[1] for d in decs):
                    allowed = fa[2](decs)              # one native call per step
                else:
                    allowed = [d.allowed() for d in decs]
            ctr = [(q.uid * 4096 + q.n_samples) & 0x7FFFFFFF for q in sample_seqs]
        # a step that fits a captured bucket replays its hipGraph (prefix
        # copy-on-write, cascade and split-KV attention included)
        use_graph = (self.graphs is not None and T <= self.graphs.buckets[-1] and T <= _GRAPH_MAX_T
                     and self.temperature == self.graphs.temperature)
        cascade = pre_tokens > 0
        # split-KV for few long-context decode sequences (K6), over the keys
        # each sequence attends itself (after the cascade prefix, if any)
        own_keys = [e[2] + e[1] - (e[4] if cascade else 0) for e in entries]
        kv_splits = choose_kv_splits(
            [e[1] for e in entries], own_keys,
            group, self.model.hkv, hq=self.model.hq) if self.device.type == "cuda" else 1
        with span("sched.pack"):
            host, layout = pack_step(entries, BLOCK_SIZE, group, copies,
                                     casc.blocks[:casc_keys // BLOCK_SIZE] if cascade else None,
                                     pre_tokens if cascade else 0, allowed, ctr)
            # layout extras: split factor, (hipGraph padding flag), longest own
            # key span in tiles (the decode kernel's own-span grid)
            own_tiles = -(-max(own_keys, default=0) // BLOCK_SIZE)
            layout = list(layout) + [kv_splits, 0, own_tiles]
            if kv_splits > 1:
                self.stats["kv_split_steps"] += 1
        t0 = time.perf_counter()
        self.stats["schedule_s"] += t0 - t_sched
        tok_dev = self.graphs.run(step_from_host(host, layout), copies, kv_splits) \
            if use_graph else None
        if tok_dev is not None:            # replayed hipGraph: forward + sampling
            self.stats["graph_steps"] += 1
            self.stats["graph_cow_steps"] += bool(copies)
            self.stats["graph_split_steps"] += kv_splits > 1
            self.stats["graph_cascade_steps"] += cascade
            self.stats["samples"] += len(sample_seqs)
            with span("launch.fetch"):
                tokens, event = self._fetch(tok_dev[:len(sample_seqs)])
        else:
            hidden, dstep = self._launch(host, layout)
            tok_dev = self._sample(hidden, dstep, len(sample_seqs))
            tokens, event = self._fetch(tok_dev) if tok_dev is not None else (None, None)
        self.stats["launch_s"] += time.perf_counter() - t0
        if self.graphs is not None:
            self.stats["graph_captures"] = self.graphs.captures
            self.stats["graph_capture_s"] = round(self.graphs.capture_s, 3)
        self.stats["tokens"] += T
        self.stats["steps"] += 1
        self.steps += 1
        return _Launch(batch_seqs, sample_seqs, tokens, event, T, tok_dev=tok_dev)

    # ------------------------------------------------------ decision lookahead
    LOOKAHEAD_MAX_SEQS = int(os.environ.get("MCP_LOOKAHEAD_MAX_SEQS", "8"))
    # queued requests join a lookahead step instead of ending lookahead (an
    # arrival would otherwise wait behind the step already queued)
    LOOKAHEAD_ADMIT = os.environ.get("MCP_LOOKAHEAD_ADMIT", "1") == "1"

    def _look_eligible(self, seqs, allow_waiting: bool = False) -> bool:
        """Every running request is at a pending grammar choice (nothing else
        to schedule), few of them, native decoders, nothing queued (or, with
        ``allow_waiting``, queued requests the next step admits)."""
        if (not seqs or len(seqs) > self.LOOKAHEAD_MAX_SEQS or (self.waiting and not allow_waiting)
                or self.inflight or len(seqs) != len(self.running)):
            return False
        fa = _native_feed_advance()
        if fa is None:
            return False
        from . import native
        if not hasattr(native._RT, "branches"):
            return False
        for q in seqs:
            if (q.is_prefix_job or q.evicted or q.pending or q.done or type(q.decoder) is not fa[1]
                    or q.decoder.done):
                return False
        return True

    def _look_start(self, L: _Launch) -> bool:
        """After a normal launch whose every sequence samples: count its
        tokens now and launch the next step over the outcomes of its samples.
        False: not eligible (the caller retires ``L`` as usual)."""
        if (L.tok_dev is None or not L.sample_seqs or len(L.sample_seqs) != len(L.batch_seqs)
                or len(L.sample_seqs) > self.LOOKAHEAD_MAX_SEQS
                or len(L.sample_seqs) != len(self.running) or self.waiting or self.inflight):
            return False
        for q, take in L.batch_seqs:
            if take != len(q.pending) or q.is_prefix_job:
                return False
        for q, take in L.batch_seqs:
            q.num_cached += take
            del q.pending[:take]
        L.booked = True
        nxt = None
        self._look_ready_t = None             # a new lookahead run: no step boundary seen yet
        if self._look_eligible(L.sample_seqs):
            with span("engine.launch"):
                nxt = self._launch_branch(L, list(L.sample_seqs))
        if nxt is None:
            with span("engine.retire"):
                self._retire(L)
            return True
        self._look = [L, nxt]
        return True

    def _launch_branch(self, prev: _Launch, seqs, admit: bool = False) -> Optional[_Launch]:
        """Launch the step after ``prev`` for every outcome of the choices
        ``prev`` samples: sequence s gets 1 + (its longest forced span) token
        rows at its next positions; the device writes the sampled outcome's
        tokens, sizes, logit row and next allowed set (ops.branch_select).
        ``admit``: queued requests join the step with their known tokens
        (prompt suffix / prefix job) after the lookahead rows.  None when the
        step does not fit (blocks, context, step budget)."""
        try:
            return self._launch_branch_inner(prev, seqs, admit)
        finally:
            if self._deferred_free:            # the step's copy list is queued on the stream
                self.alloc.free(self._deferred_free)
                self._deferred_free = []

    def _launch_branch_inner(self, prev: _Launch, seqs, admit: bool) -> Optional[_Launch]:
        from . import native
        t_sched = time.perf_counter()
        rt = native._RT
        order = prev.seqs if prev.seqs is not None else prev.sample_seqs
        row = {id(q): i for i, q in enumerate(order)}
        max_pos = getattr(self.model.cfg, "max_pos", None)
        entries, allowed, ctr, per = [], [], [], []
        T = 0
        for q in seqs:
            brs = rt.branches(q.decoder)
            if any(b[2] for b in brs):
                # an outcome that ends the plan: a step launched for it would be
                # wasted GPU work that the next request queues behind (the
                # plan's last choice runs synchronously)
                return None
            Lm = max(len(b[1]) for b in brs)
            start = q.num_cached
            if max_pos is not None and start + Lm >= max_pos:
                return None
            need = (start + Lm + BLOCK_SIZE - 1) // BLOCK_SIZE - len(q.blocks)
            if need > 0:
                if need > self.alloc.num_free:
                    return None
                q.blocks += self.alloc.alloc(need)
            entries.append(([0] * Lm, Lm, start, q.blocks, 0, True))
            allowed.append([0] * max(1, max(len(b[3]) for b in brs)))
            ctr.append((q.uid * 4096 + q.n_samples + 1) & 0x7FFFFFFF)
            per.append((row[id(q)], T, start, Lm, brs))
            T += Lm
        if T > self.max_step_tokens:
            return None
        # admitted requests: their known tokens after the lookahead rows (no
        # cascade, no memory-pressure path: a request that does not fit waits)
        copies, explicit, tail_sets = [], [], []
        if admit and self.waiting:
            self._admit()
            ids_look = {id(q) for q in seqs}
            fa = _native_feed_advance()
            for seq in self.running:
                if id(seq) in ids_look:
                    continue
                if not seq.materialized and not seq.is_prefix_job and seq.prefix is not None \
                        and seq.prefix.computed and self.alloc.num_free > 1:
                    self._materialize(seq, copies)
                if not (seq.materialized or seq.is_prefix_job) or seq.evicted or not seq.pending:
                    continue
                take = min(len(seq.pending), self.max_step_tokens - T)
                if take <= 0:
                    break
                start = seq.num_cached
                need = (start + take + BLOCK_SIZE - 1) // BLOCK_SIZE - len(seq.blocks)
                if need > 0:
                    if need >= self.alloc.num_free:
                        continue
                    seq.blocks += self.alloc.alloc(need)
                dec = seq.decoder
                sample = take == len(seq.pending) and dec is not None and not dec.done
                entries.append((seq.pending, take, start, seq.blocks, 0, sample))
                explicit.append((seq, take, sample))
                if sample:
                    a = fa[2]([dec])[0] if fa is not None and type(dec) is fa[1] else dec.allowed()
                    allowed.append(list(a))
                    tail_sets.append(list(a))
                    ctr.append((seq.uid * 4096 + seq.n_samples) & 0x7FFFFFFF)
                T += take
        # the outcome table: header, per-outcome records, allowed-set pool, tail
        n = len(seqs)
        off = 2 + 6 * n
        tab = [n, 0] + [0] * (6 * n)
        recs, pool = [], []
        pool_base = off + sum(len(p[4]) * (4 + p[3]) for p in per)
        for i, (prow, qs, start, Lm, brs) in enumerate(per):
            tab[2 + 6 * i: 8 + 6 * i] = [prow, qs, start, Lm, len(brs), off + len(recs)]
            for tok, ids, _, nxt, _ in brs:
                recs += [tok, len(ids), pool_base + len(pool), len(nxt)] + list(ids) + [0] * (Lm - len(ids))
                pool += nxt
        tab += recs + pool
        if tail_sets:
            tab[1] = len(tab)
            rel = [0]
            for a in tail_sets:
                rel.append(rel[-1] + len(a))
            tab += [len(tail_sets)] + rel + [x for a in tail_sets for x in a]
        group = self.model.cfg.group
        own_keys = [p[2] + p[3] for p in per] + [seq.num_cached + take for seq, take, _ in explicit]
        q_lens = [p[3] for p in per] + [take for _, take, _ in explicit]
        kv_splits = choose_kv_splits(q_lens, own_keys, group, self.model.hkv,
                                     hq=self.model.hq) if self.device.type == "cuda" else 1
        host, layout = pack_step(entries, BLOCK_SIZE, group, copies, None, 0, allowed, ctr)
        own_tiles = -(-max(own_keys) // BLOCK_SIZE)
        layout = list(layout) + [kv_splits, 0, own_tiles]
        tab_dev = self._look_stager.to_device(np.asarray(tab, dtype=np.int32))
        if self._look_err is None:
            self._look_err = torch.zeros(1, dtype=torch.int32, device=self.device)
        prev_tok, err = prev.tok_dev, self._look_err

        def select(dstep):
            ops.branch_select(prev_tok, tab_dev, n, dstep, err)

        t0 = time.perf_counter()
        self.stats["schedule_s"] += t0 - t_sched
        use_graph = (self.graphs is not None and T <= self.graphs.buckets[-1] and T <= _GRAPH_MAX_T
                     and self.temperature == self.graphs.temperature)
        tok_dev = self.graphs.run(step_from_host(host, layout), copies, kv_splits, pre=select) \
            if use_graph else None
        R = n + len(tail_sets)
        if tok_dev is not None:
            self.stats["graph_steps"] += 1
            self.stats["graph_cow_steps"] += bool(copies)
            self.stats["graph_split_steps"] += kv_splits > 1
            self.stats["samples"] += R
            tokens, event = self._fetch(tok_dev[:R])
        else:
            hidden, dstep = self._launch(host, layout, pre=select)
            tok_dev = self._sample(hidden, dstep, R)
            tokens, event = self._fetch(tok_dev)
        # the admitted requests' tokens are counted now (a prefix job whose
        # tokens are all queued is complete for every later step)
        for seq, take, _ in explicit:
            seq.num_cached += take
            del seq.pending[:take]
            if seq.is_prefix_job and not seq.pending:
                self._finish(seq)
        if any(q.done for q, _, _ in explicit):
            self.running = [s for s in self.running if not s.done]
        smp = [q for q, _, sm in explicit if sm]
        self.stats["lookahead_admitted"] += len(explicit)
        self.stats["launch_s"] += time.perf_counter() - t0
        self.stats["tokens"] += T
        self.stats["steps"] += 1
        self.stats["lookahead_steps"] += 1
        self.steps += 1
        return _Launch([], list(seqs) + smp, tokens, event, T, booked=True, tok_dev=tok_dev,
                       seqs=list(seqs) + smp,
                       branches=[{b[0]: b for b in p[4]} for p in per] + [None] * len(smp))

    def _wait_tokens(self, L: _Launch) -> list:
        t1 = time.perf_counter()
        with span("retire.wait"):
            if L.event is not None:
                if _SPIN_WAIT:
                    while not L.event.query():
                        pass
                else:
                    L.event.synchronize()
            toks = L.tokens.tolist() if L.tokens is not None else []
        self.stats["sample_s"] += time.perf_counter() - t1
        return toks

    # Lookahead hold (MCP_LOOKAHEAD_HOLD, default on).
    # Launching the branch step as soon as the older samples are read queues a
    # whole step ahead of any request that arrives while the current one runs:
    # at 20 intents/s that took TTFT from 4.9 to 12.2 ms.  Instead the launch
    # waits until MCP_LOOKAHEAD_LEAD_US before the current step's measured end,
    # pumping the driver's arrivals (``poll_arrivals``) meanwhile; an arrival
    # ends the wait and joins the branch step (MCP_LOOKAHEAD_ADMIT), so it
    # starts right behind the current step - where the synchronous engine
    # would start it - and the launch still overlaps the GPU.
    LOOK_HOLD = os.environ.get("MCP_LOOKAHEAD_HOLD", "1") == "1"
    LOOK_LEAD_S = float(os.environ.get("MCP_LOOKAHEAD_LEAD_US", "400")) * 1e-6

    def _look_hold(self, cur: _Launch, t_ready: float, blocked: bool):
        """Step-time bookkeeping, then the hold before ``cur``'s successor is
        launched.  ``t_ready``: when the older launch's samples were read;
        ``blocked``: the host waited for them, so the device had just finished
        that step and started ``cur`` (steps run back to back)."""
        prev, self._look_ready_t = self._look_ready_t, (t_ready if blocked else None)
        if blocked and prev is not None:
            d = t_ready - prev                  # one step, device-bound
            self._look_step_s = d if self._look_step_s == 0.0 else 0.8 * self._look_step_s + 0.2 * d
        if not (self.LOOK_HOLD and blocked and self.poll_arrivals is not None
                and self._look_step_s > 0.0) or self.waiting:
            return
        deadline = t_ready + self._look_step_s - self.LOOK_LEAD_S
        held = time.perf_counter()
        while time.perf_counter() < deadline:
            if self.poll_arrivals() or self.waiting or (cur.event is not None and cur.event.query()):
                break
            time.sleep(50e-6)
        self.stats["look_hold_s"] = self.stats.get("look_hold_s", 0.0) + time.perf_counter() - held

    def _look_device_errors(self) -> str:
        """branch_select's device error word (rows whose sampled token matched
        no outcome), read on the host's mismatch path only - a read per step
        would add a device sync - then cleared."""
        if self._look_err is None:
            return ""
        n = int(self._look_err.item())
        self._look_err.zero_()
        self.stats["lookahead_device_errors"] = self.stats.get("lookahead_device_errors", 0) + n
        return f" (device error word: {n})"

    def _step_look(self) -> int:
        """Lookahead steady state: read the older launch's samples, resolve
        the branch launch's outcome per sequence (adopt that outcome's
        decoder, count its tokens), then launch the next branch step before
        the GPU finishes the current one - or leave lookahead, retiring the
        branch launch the normal way."""
        old, cur = self._look
        t_w = time.perf_counter()
        toks = self._wait_tokens(old)
        t2 = time.perf_counter()
        blocked = t2 - t_w > 50e-6
        order = old.seqs if old.seqs is not None else old.sample_seqs
        row = {id(q): i for i, q in enumerate(order)}
        now = None
        finished = []
        bad = False
        with span("retire.update"):
            for q, brs in zip(cur.seqs, cur.branches):
                if brs is None:               # admitted with known tokens (counted at launch)
                    continue
                t = toks[row[id(q)]]
                br = brs.get(t)
                if br is None:
                    # cannot happen with the grammar's allowed sets (the kernel
                    # samples only from them); if it does, the branch step ran
                    # this request on outcome 0's tokens: fail THIS request
                    # (its blocks come back) and leave lookahead below - the
                    # host check is authoritative (branch_select's device
                    # error word marks the same case)
                    q.error = (f"decision lookahead: sampled token {t} is not an outcome "
                               f"of the pending choice{self._look_device_errors()}")
                    finished.append(q)
                    bad = True
                    continue
                tok, ids, fin, _, dec = br
                if q.t_first is None:
                    q.t_first = now = now or time.perf_counter()
                q.n_samples += 1
                q.decoder = dec
                q.tokens += ids
                if fin:
                    finished.append(q)
                else:
                    q.num_cached += len(ids)
            for q in finished:
                self._finish(q)             # its blocks' later writers queue after this step
            if finished:
                self.running = [s for s in self.running if not s.done]
        self.stats["update_s"] += time.perf_counter() - t2
        live = [q for q in cur.seqs if not q.done]
        nxt = None
        if live and not bad:
            self._look_hold(cur, t2, blocked)
        if live and not bad and self._look_eligible(live, allow_waiting=self.LOOKAHEAD_ADMIT):
            with span("engine.launch"):
                nxt = self._launch_branch(cur, live, admit=self.LOOKAHEAD_ADMIT)
        if nxt is not None:
            self._look = [cur, nxt]
        else:
            self._look = []
            ctoks = self._wait_tokens(cur)
            rows = [i for i, q in enumerate(cur.seqs) if not q.done]
            seqs = [cur.seqs[i] for i in rows]
            t3 = time.perf_counter()
            with span("retire.update"):
                self._update([(q, 0) for q in seqs], seqs, [ctoks[i] for i in rows], booked=True)
            self.stats["update_s"] += time.perf_counter() - t3
        self.last_progress = time.perf_counter()
        return old.T + 1

    def _retire(self, L: _Launch):
        """Wait for a launch's sampled tokens and advance its sequences."""
        t1 = time.perf_counter()
        with span("retire.wait"):
            if L.event is not None:
                if _SPIN_WAIT:
                    # poll: the host picks the sampled tokens up as soon as the
                    # copy lands instead of after hipEventSynchronize's wake-up
                    ev = L.event
                    while not ev.query():
                        pass
                else:
                    L.event.synchronize()
            new_tokens = L.tokens.tolist() if L.tokens is not None else []
        t2 = time.perf_counter()
        self.stats["sample_s"] += t2 - t1
        if self.bcast is not None:          # TP: a collective that timed out fails the step
            self.model.comm_check()
        batch_seqs, sample_seqs = L.batch_seqs, L.sample_seqs
        with span("retire.update"):
            self._update(batch_seqs, sample_seqs, new_tokens, booked=L.booked)
        self.stats["update_s"] += time.perf_counter() - t2
        METRICS.set("batch_occupancy", len(self.running))
        METRICS.set("kv_block_utilization", self.alloc.utilization())

    def _update(self, batch_seqs, sample_seqs, new_tokens, booked: bool = False):
        # ---- bookkeeping (a lookahead launch counted its tokens at launch)
        for seq, take in ([] if booked else batch_seqs):
            seq.num_cached += take
            del seq.pending[:take]
            if seq.is_prefix_job and not seq.pending:
                self._finish(seq)
        decs = [seq.decoder for seq in sample_seqs]
        fa = _native_feed_advance()
        if fa is not None and decs and all(type(d) is fa[1] for d in decs):
            news = fa[0](decs, new_tokens)          # native decoders: one call per step
        else:
            news = []
            for d, tok in zip(decs, new_tokens):
                d.feed(int(tok))
                news.append(d.advance())
        now = None
        for seq, new in zip(sample_seqs, news):
            if seq.t_first is None:
                seq.t_first = now = now or time.perf_counter()
            seq.n_samples += 1
            seq.pending += new
            seq.tokens += new
        max_pos = getattr(self.model.cfg, "max_pos", None)
        for seq, _ in batch_seqs:
            if seq.is_prefix_job or seq.done:
                continue
            if seq.decoder.done:
                self._finish(seq)
            elif max_pos is not None and seq.num_cached + len(seq.pending) >= max_pos:
                # the grammar's output does not fit the context left: fail the
                # request instead of running positions past the RoPE table
                seq.error = (f"context exhausted: the plan reached the model's {max_pos}-token "
                             f"limit ({seq.num_cached} cached + {len(seq.pending)} pending)")
                self._finish(seq)
        self.running = [s for s in self.running if not s.done]

    def _launch(self, host, layout, pre=None):
        """(packed step) -> (broadcast to TP workers) -> H2D -> KV copies ->
        (``pre``: the lookahead's outcome selection) -> forward."""
        with span("launch.h2d"):
            payload = self.stager.to_device(host)
        if self.bcast is not None:
            self.bcast.send(payload, layout)
        dstep, csrc, cdst = views(payload, layout)
        if pre is not None:
            pre(dstep)
        if csrc.numel():
            ops.copy_blocks(self.kv.data, csrc, cdst)
        if dstep.token_ids.numel() == 0:
            return None, dstep
        with span("launch.forward"):
            return self.model.forward(dstep, self.kv), dstep

    def shutdown_workers(self):
        if self.bcast is not None:
            self.bcast.stop()

    def _sample(self, hidden: torch.Tensor, dstep, n: int) -> Optional[torch.Tensor]:
        """Fused LM-head-rows + grammar mask + Gumbel-max sampling (K9) on the
        allowed sets that travelled with the step descriptor.  The RNG counter
        (request uid, sample index) makes every draw unique, so the seed is
        constant (the same kernel runs inside captured hipGraphs)."""
        if n == 0:
            return None
        tok = ops.sample_allowed(hidden, self.model.w.lm_head, dstep.allow_ptr, dstep.allow_ids,
                                 dstep.sample_ctr, self.temperature, self.seed)
        self.stats["samples"] += n
        return tok

    @staticmethod
    def _fetch(tok: torch.Tensor):
        """Async D2H of sampled tokens into pinned memory + completion event."""
        if tok.numel() == 0:
            return None, None
        if not tok.is_cuda:
            return tok, None
        host = torch.empty(tok.numel(), dtype=torch.int32, pin_memory=True)
        host.copy_(tok, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return host, ev

    def warm_graphs(self, max_tokens: Optional[int] = None, contexts=(2048,)) -> int:
        """Capture the hipGraph buckets ahead of serving (server start-up);
        0 when graphs are off."""
        if self.graphs is None:
            return 0
        max_tokens = _GRAPH_MAX_T if max_tokens is None else min(max_tokens, _GRAPH_MAX_T)
        return self.graphs.warm(max_tokens, contexts)

    # -------------------------------------------------------------- driver
    def run(self, max_steps: int = 1_000_000):
        n = idle = 0
        while self.has_work() and n < max_steps:
            if self.step() == 0 and not self.inflight and not self._look:
                if not self.waiting:
                    # nothing runnable: sequences blocked on nothing -> bug guard
                    stuck = [s for s in self.running if not s.pending]
                    if stuck:
                        raise RuntimeError("engine stalled with sequences that have no pending tokens")
                # a step without progress may release blocks for the next one;
                # several in a row with nothing in flight can never progress
                idle += 1
                if idle > 8:
                    raise RuntimeError(f"engine stalled: {len(self.running)} running and "
                                       f"{len(self.waiting)} waiting requests cannot be scheduled "
                                       f"({self.alloc.num_free} of {self.kv.num_blocks} KV blocks free)")
            else:
                idle = 0
            n += 1
        return n
