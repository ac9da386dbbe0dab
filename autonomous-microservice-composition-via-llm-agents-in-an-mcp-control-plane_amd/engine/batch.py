"""Per-step batch metadata (host side) for the ragged, paged forward pass.

One engine step feeds a ragged batch: sequence ``s`` contributes ``q_len[s]``
new tokens (1 for decode, a chunk for prefill / grammar jump-forward) whose KV
lands in the paged cache, and attends causally to ``ctx_len[s]`` keys.

All int32 metadata of a step is packed into ONE host buffer and moved with ONE
host->device copy (``pack``); the attention work lists are derived here too:
sequences with few new tokens go to the 1-wave kernel variant, longer ones to
the 4-wave variant (csrc/attention.hip).
"""
from __future__ import annotations

import dataclasses
import os
from typing import List, Optional, Sequence

import numpy as np
import torch

BLOCK_SIZE = 64


def tokens_per_item(nw: int, group: int) -> int:
    return nw * (16 // group)


@dataclasses.dataclass
class AttnMeta:
    q_start: torch.Tensor      # [S] int32
    q_len: torch.Tensor        # [S]
    ctx_len: torch.Tensor      # [S]
    block_table: torch.Tensor  # [S, max_blocks]
    work: List[tuple]          # [(nw, work_seq[int32], work_q0[int32]), ...]
    # cascade attention over one shared prefix (None when unused):
    kv_begin: Optional[torch.Tensor] = None   # [S] first key each sequence attends itself
    pre_bt: Optional[torch.Tensor] = None     # block ids of the shared prefix
    pre_keys: int = 0                         # shared prefix keys (multiple of 64)
    pre_tokens: int = 0                       # flat tokens [0, pre_tokens) attend to it
    kv_splits: int = 1                        # split-KV factor of the 1-wave items (K6)
    # hipGraph static layout: the work lists are padded to the key's capacity
    # (their lengths are not the step's item counts)
    padded: bool = False
    # hipGraph steps: device [pre_tokens, pre_keys] (the host ints above are
    # then the bucket's capacities, engine/graphs.py)
    pre_dims: Optional[torch.Tensor] = None
    # longest own key span of the step in 64-key tiles (keys after the cascade
    # prefix); 0 = unknown (hipGraph layouts)
    own_tiles: int = 0

    def work_lists(self):
        return self.work


_XCD_ORDER = os.environ.get("MCP_ATTN_XCD_ORDER", "1") == "1"
# fewest own key tiles (of the longest sequence) for a split-KV step.  4
# (was 8): serving steps of a few requests with 4-7 own key tiles each split
# too - config 5 at 40 intents/s p50 172-178 -> 147-150 ms, 80/s 213-221 ->
# 202-213 ms, 20/s 123 -> 119-121 ms (same box; 2 measured equal to 4,
# profiles/attention_splitkv_min_tiles_ab.jsonl).  MCP_KV_SPLIT_MIN_TILES overrides
_SPLIT_MIN_TILES = int(os.environ.get("MCP_KV_SPLIT_MIN_TILES", "4"))
# split only while the step has fewer than this many x num_cus work items:
# 2 (was 1) - config 5 at 80 intents/s p50 195-196 -> 188-190 ms, p99 244 ->
# 230, 120/s 321-333 -> 316-321 (profiles/attention_splitkv_min_tiles_ab.jsonl)
_SPLIT_WORK_FACTOR = float(os.environ.get("MCP_KV_SPLIT_WORK_FACTOR", "2"))
_SPLIT_SHORT = os.environ.get("MCP_KV_SPLIT_SHORT", "0") == "1"
N_SIZES = 19            # packed segments of pack_host (the layout's leading entries)


def choose_kv_splits(q_lens, kv_lens, group: int, hkv: int, num_cus: int = 256,
                     max_bytes: int = 64 << 20, hq: int = 32) -> int:
    """Split-KV factor for the attention items of a step (csrc/attention.hip
    KSPLIT, 1-wave and 4-wave items).  A step of few sequences with long
    contexts has few work items (one per sequence and kv head) on 256 CUs -
    batch-1 decode on 8B is 8 workgroups walking the whole context.  Split each
    item's own key range (``kv_lens`` = keys it attends itself, after any
    cascade prefix) so the grid reaches ~2 workgroups per CU (prefill chunks
    make enough items and are never split).
    ``MCP_KV_SPLIT``: 0 disables, N > 1 forces N."""
    forced = int(os.environ.get("MCP_KV_SPLIT", "-1"))
    if forced == 0:
        return 1
    if forced < 0 and sum(1 for ql in q_lens if ql > 0) * hkv >= _SPLIT_WORK_FACTOR * num_cus:
        # every sequence is at least one work item per kv head: never split
        # (the per-step host path skips the loop below for large batches)
        return 1
    t1 = tokens_per_item(1, group)
    t4 = tokens_per_item(4, group)
    cutoff = int(os.environ.get("MCP_ATTN_NW1_CUTOFF", str(t1 * 2)))
    items, tiles, rows = 0, 0, 0
    for ql, kl in zip(q_lens, kv_lens):
        if ql <= 0:
            continue
        # 1-wave items (decode) and 4-wave items (jump-forward spans) both split
        items += -(-ql // t1) if ql <= cutoff else -(-ql // t4)
        tiles = max(tiles, -(-kl // 64))
        rows += ql
    if items == 0:
        return 1
    if forced > 1:
        return forced
    work = items * hkv
    if work >= _SPLIT_WORK_FACTOR * num_cus or tiles < _SPLIT_MIN_TILES:
        return 1
    # ~2 workgroups per CU (measured best at batch 1 / 4 and 8k-128k contexts,
    # profiles/attention_splitkv.jsonl); >= 4 key tiles per split there, >= 2
    # for the ~700-1000-key contexts of a single intent (config 2: 4-8 splits
    # of 11-16 tiles measured 113 ms p50 vs 119 unsplit)
    # Round 6: short contexts (< 16 own tiles) with decode-sized query spans
    # (<= 8 rows each) split down to ONE tile per split - one sequence, 700
    # keys, 1-8 new tokens: 8 splits 10.6-12.0 us against 4 splits 12.3-13.2
    # (tools/bench_attention_decode.py, profiles/attention_decode_r6.jsonl);
    # with 16-row spans 4 splits stay ahead.  End to end it measured neutral
    # (config 2 p50 85.3-85.7 vs 84.5-85.3 ms, config 5 at 20 / 40 intents/s
    # +0.8 / -0.7 ms; profiles/kv_split_short_ab_r6.txt): MCP_KV_SPLIT_SHORT=1
    # turns it on, default off.
    per = 4 if tiles >= 32 else 2
    if tiles < 16 and _SPLIT_SHORT and max(q_lens) <= 8:
        per = 1
    ns = min(tiles // per, -(-2 * num_cus // work), 128)
    sum_tokens = max(sum(q_lens), 1)
    while ns > 1 and ns * sum_tokens * hq * 128 * 4 > max_bytes:
        ns //= 2
    # a power of two: the split count is part of the hipGraph key, and a
    # handful of values can all be captured at start-up (engine/graphs.py)
    p2 = 1
    while p2 * 2 <= ns:
        p2 *= 2
    return p2


def build_work(q_len: Sequence[int], group: int, small_cutoff: Optional[int] = None):
    """Split each sequence's query span into work items.

    Returns {nw: (seq_ids, q0s)} with nw in {1, 4}."""
    t1 = tokens_per_item(1, group)
    t4 = tokens_per_item(4, group)
    if small_cutoff is None:
        small_cutoff = int(os.environ.get("MCP_ATTN_NW1_CUTOFF", str(t1 * 2)))
    cutoff = small_cutoff
    out = {1: ([], []), 4: ([], [])}
    for s, ql in enumerate(q_len):
        if ql <= 0:
            continue
        nw, qt = (1, t1) if ql <= cutoff else (4, t4)
        for q0 in range(0, ql, qt):
            out[nw][0].append(s)
            out[nw][1].append(q0)
    if _XCD_ORDER and out[1][0]:
        # 1-wave items of one sequence read the same K/V: place them 8 work
        # slots apart so they land on one XCD (block id % 8) and share its L2
        # (sequences bucketed by item count, deepest first, so that a block of
        # 8 sequences has equal depth and item d of sequence i sits at 8 d + i)
        seqs, q0s = out[1]
        groups = {}
        for sq, q0 in zip(seqs, q0s):
            groups.setdefault(sq, []).append(q0)
        rs, rq = [], []
        for depth in sorted({len(v) for v in groups.values()}, reverse=True):
            order = [x for x in groups if len(groups[x]) == depth]
            for b in range(0, len(order), 8):
                blk = order[b:b + 8]
                for d in range(depth):
                    for x in blk:
                        rs.append(x)
                        rq.append(groups[x][d])
        out[1] = (rs, rq)
    return out


@dataclasses.dataclass
class StepInputs:
    """Host-side description of one forward step."""
    token_ids: np.ndarray      # [T] int32
    positions: np.ndarray      # [T] int32
    slots: np.ndarray          # [T] int32 (physical KV slot, -1 = skip)
    q_start: np.ndarray        # [S]
    q_len: np.ndarray          # [S]
    ctx_len: np.ndarray        # [S]
    block_table: np.ndarray    # [S, max_blocks]
    logit_rows: np.ndarray     # [R] token row whose hidden feeds sampling
    kv_begin: Optional[np.ndarray] = None   # [S] cascade: first own key per sequence
    pre_bt: Optional[np.ndarray] = None     # cascade: shared prefix blocks
    pre_tokens: int = 0                     # cascade: leading flat tokens that share it
    allow_ptr: Optional[np.ndarray] = None  # [R+1] sampling: CSR of grammar-allowed tokens
    allow_ids: Optional[np.ndarray] = None  # [A]
    sample_ctr: Optional[np.ndarray] = None  # [R] RNG counters

    @property
    def num_tokens(self) -> int:
        return int(self.token_ids.shape[0])


@dataclasses.dataclass
class DeviceStep:
    token_ids: torch.Tensor
    positions: torch.Tensor
    slots: torch.Tensor
    logit_rows: torch.Tensor
    attn: AttnMeta
    allow_ptr: Optional[torch.Tensor] = None
    allow_ids: Optional[torch.Tensor] = None
    sample_ctr: Optional[torch.Tensor] = None


def pack_host(step: StepInputs, group: int, copies=()):
    """All int32 metadata of one step (+ prefix copy-on-write block pairs) in
    ONE host array; ``layout`` = the segment sizes (also what TP workers need)."""
    work = build_work(step.q_len.tolist(), group)
    cp = np.asarray(copies, np.int32).reshape(-1, 2) if len(copies) else np.zeros((0, 2), np.int32)
    parts = [step.token_ids, step.positions, step.slots, step.logit_rows, step.q_start,
             step.q_len, step.ctx_len, step.block_table.reshape(-1)]
    for nw in (1, 4):
        parts += [np.asarray(work[nw][0], np.int32), np.asarray(work[nw][1], np.int32)]
    parts += [cp[:, 0].copy(), cp[:, 1].copy()]
    S = int(step.q_len.shape[0])
    cascade = step.pre_bt is not None and step.pre_tokens > 0 and len(step.pre_bt) > 0
    parts += [step.kv_begin if cascade else np.zeros(0, np.int32),
              np.asarray(step.pre_bt, np.int32) if cascade else np.zeros(0, np.int32)]
    z = np.zeros(0, np.int32)
    parts += [step.allow_ptr if step.allow_ptr is not None else z,
              step.allow_ids if step.allow_ids is not None else z,
              step.sample_ctr if step.sample_ctr is not None else z]
    layout = [int(p.size) for p in parts] + [S, int(step.pre_tokens) if cascade else 0]
    host = np.concatenate([np.asarray(p, dtype=np.int32).reshape(-1) for p in parts]) \
        if sum(layout[:-1]) else np.zeros(0, np.int32)
    return host, layout


class HostStager:
    """Persistent pinned host staging for the per-step H2D copy.

    Two pinned int32 buffers alternate; before one is reused the event recorded
    after its last async copy is waited on (in steady state it completed long
    ago, because every step synchronises on the sampled tokens)."""

    def __init__(self, device):
        self.device = torch.device(device) if device is not None else None
        self._buf = [None, None]
        self._ev = [None, None]
        self._i = 0

    def to_device(self, host: np.ndarray, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Async H2D of ``host``; into ``out`` (a static device buffer) when given."""
        if self.device is None or self.device.type != "cuda":
            t = torch.from_numpy(host)
            return t if out is None else out[:t.numel()].copy_(t)
        i = self._i
        self._i ^= 1
        n = int(host.size)
        b = self._buf[i]
        if self._ev[i] is not None:
            self._ev[i].synchronize()
        if b is None or b.numel() < n:
            b = torch.empty(max(n, 2 * (b.numel() if b is not None else 4096)), dtype=torch.int32,
                            pin_memory=True)
            self._buf[i] = b
        np.copyto(b.numpy()[:n], host)
        if out is not None:
            d = out[:n]
            d.copy_(b[:n], non_blocking=True)
        else:
            d = b[:n].to(self.device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._ev[i] = ev
        return d


def pack_step_py(entries, block_size: int, group: int, copies=None, pre_bt=None, pre_tokens: int = 0,
                 allowed=None, ctr=None):
    """Python reference of the native ``pack_step`` (csrc/runtime/runtime.cpp).

    ``entries``: (tokens, take, start, blocks, kv_begin, sample) per sequence;
    the first ``take`` tokens enter at positions [start, start + take).
    Returns ``(host, layout)`` like ``pack_host``."""
    ids, pos, slots, rows = [], [], [], []
    q_start, q_len, ctx_len, kvb, tables = [], [], [], [], []
    T = 0
    for toks, take, start, blocks, kv_begin, sample in entries:
        if take <= 0 or take > len(toks):
            raise ValueError("pack_step: bad span")
        if start + take > len(blocks) * block_size:
            raise ValueError("pack_step: sequence has too few KV blocks")
        ids += list(toks[:take])
        p = np.arange(start, start + take, dtype=np.int32)
        pos.append(p)
        blk = np.asarray(blocks, dtype=np.int32)
        slots.append(blk[p // block_size] * block_size + p % block_size)
        q_start.append(T)
        q_len.append(take)
        ctx_len.append(start + take)
        kvb.append(kv_begin)
        tables.append(blocks)
        T += take
        if sample:
            rows.append(T - 1)
    S = len(entries)
    maxb = max([len(t) for t in tables] + [1])
    bt = np.zeros((S, maxb), np.int32)
    for i, t in enumerate(tables):
        bt[i, :len(t)] = t
    z = np.zeros(0, np.int32)
    step = StepInputs(token_ids=np.asarray(ids, np.int32),
                      positions=np.concatenate(pos) if pos else z,
                      slots=np.concatenate(slots).astype(np.int32) if slots else z,
                      q_start=np.asarray(q_start, np.int32), q_len=np.asarray(q_len, np.int32),
                      ctx_len=np.asarray(ctx_len, np.int32), block_table=bt,
                      logit_rows=np.asarray(rows, np.int32))
    if pre_bt is not None and pre_tokens > 0 and len(pre_bt):
        step.kv_begin = np.asarray(kvb, np.int32)
        step.pre_bt = np.asarray(pre_bt, np.int32)
        step.pre_tokens = pre_tokens
    if allowed is not None:
        ptr = np.zeros(len(allowed) + 1, np.int32)
        ptr[1:] = np.cumsum([len(a) for a in allowed])
        step.allow_ptr = ptr
        step.allow_ids = np.asarray([t for a in allowed for t in a], np.int32)
        step.sample_ctr = np.asarray(ctr, np.int32)
        if len(step.sample_ctr) != len(rows) or len(allowed) != len(rows):
            raise ValueError("pack_step: allowed sets / counters do not match sampled rows")
    return pack_host(step, group, copies or ())


def pack_step(entries, block_size: int, group: int, copies=None, pre_bt=None, pre_tokens: int = 0,
              allowed=None, ctr=None):
    """One step's packed int32 descriptor: the native C++ packer when built."""
    from . import native
    if native.available():
        return native.pack_step(entries, block_size, group, list(copies) if copies else None,
                                pre_bt, pre_tokens, allowed, ctr)
    return pack_step_py(entries, block_size, group, copies, pre_bt, pre_tokens, allowed, ctr)


def step_from_host(host: np.ndarray, layout) -> StepInputs:
    """``StepInputs`` of numpy views into a packed host buffer (the inverse of
    ``pack_host`` on the host side; used by the hipGraph bucket packer)."""
    sizes, S, pre_tokens = layout[:N_SIZES], layout[N_SIZES], layout[N_SIZES + 1]
    vs, off = [], 0
    for n in sizes:
        vs.append(host[off:off + n])
        off += n
    bt = vs[7].reshape(S, -1) if S else vs[7].reshape(0, 1)
    step = StepInputs(token_ids=vs[0], positions=vs[1], slots=vs[2], q_start=vs[4], q_len=vs[5],
                      ctx_len=vs[6], block_table=bt, logit_rows=vs[3])
    if pre_tokens > 0:
        step.kv_begin, step.pre_bt, step.pre_tokens = vs[14], vs[15], pre_tokens
    if sizes[16]:
        step.allow_ptr, step.allow_ids, step.sample_ctr = vs[16], vs[17], vs[18]
    return step


def to_device(host: np.ndarray, device, pin: bool = True) -> torch.Tensor:
    t = torch.from_numpy(host)
    if device is not None and torch.device(device).type == "cuda":
        if pin:
            t = t.pin_memory()
        t = t.to(device, non_blocking=True)
    return t


def views(t: torch.Tensor, layout):
    """Inverse of ``pack_host`` on an (already transferred) int32 tensor.
    Returns (DeviceStep, copy_src, copy_dst)."""
    sizes, S, pre_tokens = layout[:N_SIZES], layout[N_SIZES], layout[N_SIZES + 1]
    vs, off = [], 0
    for n in sizes:
        vs.append(t[off:off + n])
        off += n
    bt = vs[7].view(S, -1) if S else vs[7].view(0, 1)
    work_l = []
    for i, nw in enumerate((1, 4)):
        ws, wq = vs[8 + 2 * i], vs[9 + 2 * i]
        if ws.numel():
            work_l.append((nw, ws, wq))
    meta = AttnMeta(q_start=vs[4], q_len=vs[5], ctx_len=vs[6], block_table=bt, work=work_l,
                    kv_splits=int(layout[N_SIZES + 2]) if len(layout) > N_SIZES + 2 else 1,
                    padded=len(layout) > N_SIZES + 3 and bool(layout[N_SIZES + 3]),
                    own_tiles=int(layout[N_SIZES + 4]) if len(layout) > N_SIZES + 4 else 0)
    if pre_tokens > 0:
        meta.kv_begin, meta.pre_bt = vs[14], vs[15]
        meta.pre_keys, meta.pre_tokens = int(vs[15].numel()) * BLOCK_SIZE, pre_tokens
    elif pre_tokens < 0:
        # static (hipGraph) layout: segment 15 = [pre_tokens, pre_keys, blocks...]
        # read on the device; capacities: the step's token count and the blocks
        meta.kv_begin, meta.pre_dims, meta.pre_bt = vs[14], vs[15][:2], vs[15][2:]
        meta.pre_keys, meta.pre_tokens = int(vs[15].numel() - 2) * BLOCK_SIZE, int(vs[0].numel())
    d = DeviceStep(token_ids=vs[0], positions=vs[1], slots=vs[2], logit_rows=vs[3], attn=meta)
    d.allow_ptr, d.allow_ids, d.sample_ctr = vs[16], vs[17], vs[18]
    return d, vs[12], vs[13]


def pack(step: StepInputs, group: int, device, pin: bool = True) -> DeviceStep:
    """Pack all int32 arrays into one buffer -> one H2D copy -> views."""
    host, layout = pack_host(step, group)
    return views(to_device(host, device, pin), layout)[0]
