"""Process groups and collectives (collective sites C1-C5).

One process per GPU; ``torch.distributed`` with backend ``"nccl"`` is RCCL on
ROCm and runs over xGMI between the 8 MI355X of a node.  The CPU test tier
uses ``gloo`` with the same code paths.

* ``init_distributed``  – env:// rendezvous (torchrun), binds the local GPU.
* ``NativeComm``        – K13: an RCCL communicator driven directly through
  ``rccl.h`` (``csrc/rccl_comm.hip``) on the caller's HIP stream; the
  ncclUniqueId is bootstrapped over the torch process group (C5).
* ``AllReduce``         – in-place sum for the row-parallel projections
  (C1 after Wo, C2 after Wdown).  GPU: the xGMI peer-to-peer kernel of
  ``parallel.custom_allreduce`` for decode-sized messages (default on), the
  native RCCL communicator above its size limit (``MCP_COMM=native``,
  default) or torch.distributed's (``MCP_COMM=torch``); CPU: gloo in fp32.
* ``StepBroadcaster``   – C4: the driver rank broadcasts each step's packed
  int32 descriptor (tokens, positions, slots, block tables, work lists, KV
  copy-on-write pairs) to the TP worker ranks.
"""
from __future__ import annotations

import os
from typing import Callable, Optional

import numpy as np
import torch
import torch.distributed as dist


def init_distributed(backend: Optional[str] = None):
    """Returns (rank, world_size, local_rank, device)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available() and backend != "gloo"
    device = torch.device("cuda", local_rank) if use_gpu else torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        if use_gpu:
            torch.cuda.set_device(local_rank)
            dist.init_process_group(backend or "nccl", device_id=device)
        else:
            dist.init_process_group(backend or "gloo")
    return rank, world, local_rank, device


class NativeComm:
    """Direct RCCL communicator over the ranks of ``group``."""

    OPS = {"sum": 0, "max": 1, "min": 2}

    def __init__(self, group, device):
        from .. import ops
        self._lib = ops.lib()
        self.device = torch.device(device)
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        obj = [self._lib.nccl_unique_id().numpy().tobytes() if self.rank == 0 else None]
        dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None
                                   else 0, group=group)
        uid = torch.frombuffer(bytearray(obj[0]), dtype=torch.uint8).clone()
        with torch.cuda.device(self.device):
            self._comm = self._lib.nccl_init(self.world, self.rank, uid)

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        self._lib.nccl_all_reduce(self._comm, t, self.OPS[op])
        return t

    def all_gather(self, t: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        out = t.new_empty((self.world,) + tuple(t.shape)) if out is None else out
        self._lib.nccl_all_gather(self._comm, t.contiguous(), out)
        return out

    def reduce_scatter(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        out = t.new_empty((t.numel() // self.world,))
        self._lib.nccl_reduce_scatter(self._comm, t.contiguous(), out, self.OPS[op])
        return out

    def broadcast(self, t: torch.Tensor, root: int = 0) -> torch.Tensor:
        self._lib.nccl_broadcast(self._comm, t, root)
        return t

    def close(self):
        if self._comm:
            self._lib.nccl_destroy(self._comm)
            self._comm = 0


K12_MAX_BYTES = 64 << 20       # K12 staging buffer per epoch parity (2 per rank)


class AllReduce:
    """In-place sum over the TP group for the row-parallel projections (C1, C2).

    GPU: the path the xGMI cost model (``parallel/xgmi_model.py``) prices
    lowest - K12 (``parallel.custom_allreduce``, peer reads on all links at
    once; one-shot below the model's crossover, two-shot above) for every
    message its staging buffer holds, ``MCP_CAR_MAX_BYTES`` (default 64 MiB:
    prefill steps of up to 4096 tokens at H = 8192; the model prices K12
    two-shot under RCCL at every size), the native RCCL communicator above
    that (``MCP_COMM=native``, default) or torch.distributed's
    (``MCP_COMM=torch``).  ``MCP_CUSTOM_ALLREDUCE``
    = auto (default: on for GPU groups of 2-8 ranks) | 1 | 0.
    CPU: gloo in fp32.

    ``check()`` raises when a K12 barrier timed out (a peer never arrived): the
    engine calls it after every step, so a lost peer is a hard failure instead
    of activations summed from stale staging buffers.

    Start-up self-check (``MCP_CAR_SELFCHECK=1``, default): K12's peers read
    each other's staging buffers over xGMI (coarse-grained ``hipMalloc``
    memory, system-scope flags, ``csrc/custom_allreduce.hip``).  Before the
    first real message every rank sums probe tensors of known integer values
    through K12 in both modes (one-shot and two-shot) and through the RCCL
    path, and checks both against the exact sum; the ranks agree on the
    outcome (``all_gather_object``), and a K12 mismatch on any rank disables
    K12 on every rank (all messages then take RCCL) with a logged reason
    (``custom_disabled``).  An RCCL mismatch is a hard error."""

    def __init__(self, group, device):
        self.group = group
        self.device = torch.device(device)
        self.custom = None
        self.native = None
        self.custom_disabled: Optional[str] = None
        if self.device.type != "cuda":
            return
        world = dist.get_world_size(group)
        mode = os.environ.get("MCP_CUSTOM_ALLREDUCE", "auto")
        if mode == "1" or (mode == "auto" and 2 <= world <= 8):
            from .custom_allreduce import CustomAllReduce
            self.custom = CustomAllReduce(group, self.device,
                                          max_bytes=int(os.environ.get("MCP_CAR_MAX_BYTES",
                                                                       str(K12_MAX_BYTES))))
            # the largest message the model still sends through K12 (RCCL
            # above it; at the default constants: the whole staging buffer)
            from .xgmi_model import best
            m = self.custom.max_bytes
            if best(m, world, m)[0] == "rccl":
                lo, hi = 0, m
                while hi - lo > 4096:
                    mid = (lo + hi) // 2
                    if best(mid, world, m)[0] == "rccl":
                        hi = mid
                    else:
                        lo = mid
                self.custom.max_bytes = lo
        if os.environ.get("MCP_COMM", "native") == "native":
            self.native = NativeComm(group, self.device)
        if self.custom is not None and os.environ.get("MCP_CAR_SELFCHECK", "1") == "1":
            self._selfcheck()

    def _reference_sum(self, t: torch.Tensor) -> None:
        if self.native is not None:
            self.native.all_reduce(t)
        else:
            dist.all_reduce(t, group=self.group)

    def _selfcheck(self) -> None:
        rank, world = dist.get_rank(self.group), dist.get_world_size(self.group)
        inject = os.environ.get("MCP_CAR_SELFCHECK_INJECT")   # tests: this rank's K12 result is wrong
        sizes = [n for n in (8 << 10, min(self.custom.max_bytes, 2 << 20) // 2)
                 if 0 < n * 2 <= self.custom.max_bytes]
        with torch.cuda.device(self.device):
            verdict = selfcheck_decision(
                rank, world, sizes,
                probe=lambda n, r: probe_values(n, r, self.device),
                custom=lambda t, mode: self.custom(t, mode=mode),
                reference=self._reference_sum,
                agree=lambda mine: _gather_objects(mine, self.group),
                inject=inject is not None and int(inject) == rank)
        if verdict.get("reference_error"):
            raise RuntimeError(f"all-reduce self-check: the RCCL path is wrong: {verdict}")
        if not verdict["custom_ok"]:
            import logging
            logging.getLogger("mcp.comm").warning(
                "custom all-reduce (K12) disabled: start-up self-check mismatch %s", verdict["why"])
            self.custom.close()
            self.custom = None
            self.custom_disabled = verdict["why"]

    # accepts ``ss_out`` (the fused RMSNorm statistic of the summed rows)
    supports_ss = True

    def __call__(self, t: torch.Tensor, ss_out: Optional[torch.Tensor] = None) -> None:
        """In-place sum; with ``ss_out`` (int64, zeroed) also the summed rows'
        fixed-point sums of squares - inside K12 when it takes the message
        (no extra pass), else one ``row_sumsq`` pass after the collective."""
        if self.device.type != "cuda":
            tf = t.float()
            dist.all_reduce(tf, group=self.group)
            t.copy_(tf.to(t.dtype))
        elif self.custom is not None and self.custom.eligible(t):
            if ss_out is not None and self.custom.ss_eligible(t):
                self.custom(t, ss_out=ss_out)
                return
            self.custom(t)
        elif self.native is not None:
            self.native.all_reduce(t)
        else:
            dist.all_reduce(t, group=self.group)
        if ss_out is not None:
            from .. import ops
            ops.row_sumsq(t.view(-1, t.shape[-1]), ss_out)

    def check(self) -> None:
        if self.custom is not None:
            self.custom.check()

    def graph_safe(self, nbytes: int) -> bool:
        """Whether an all-reduce of up to ``nbytes`` can be captured in a
        hipGraph: K12 (device-side epochs) and RCCL on the capture stream are;
        a gloo collective on a GPU tensor (CPU tests) is host code and is not."""
        if self.device.type != "cuda":
            return False
        if self.custom is not None and nbytes <= self.custom.max_bytes:
            return True
        return self.native is not None or not _is_gloo(self.group)


def probe_values(n: int, rank: int, device) -> torch.Tensor:
    """Self-check probe: small integers (exact in bf16, and so is their sum
    over <= 8 ranks) that differ per rank and per element."""
    i = torch.arange(n, device=device, dtype=torch.int32)
    return ((i * 7 + rank * 3) % 11 + (i % 5 == rank % 5).int() * 2).to(torch.bfloat16)


def selfcheck_decision(rank: int, world: int, sizes, probe, custom, reference, agree,
                       inject: bool = False) -> dict:
    """One rank's part of the K12 start-up self-check.  For every probe size,
    K12 one-shot (mode 1) and two-shot (mode 2) and the reference collective
    each sum ``probe(n, rank)`` over the group and are compared with the exact
    sum (computed locally from ``probe(n, r)`` of every rank).  ``agree``
    exchanges every rank's findings; K12 stays on only if no rank saw a
    mismatch.  Returns {"custom_ok", "reference_error", "why"}."""
    bad, ref_bad = [], []
    for n in sizes:
        exact = sum(probe(n, r).float() for r in range(world))
        for mode in (1, 2):
            t = probe(n, rank)
            out = custom(t, mode)
            if inject:
                out = out.clone()
                out[n // 2] += 1
            if not torch.equal(out.float(), exact):
                bad.append(f"rank {rank}: K12 mode {mode}, {n * 2} B: "
                           f"{int((out.float() != exact).sum())} wrong elements")
        t = probe(n, rank)
        reference(t)
        if not torch.equal(t.float(), exact):
            ref_bad.append(f"rank {rank}: reference all-reduce, {n * 2} B")
    every = agree({"bad": bad, "ref_bad": ref_bad})
    bad_all = [b for e in every for b in e["bad"]]
    ref_all = [b for e in every for b in e["ref_bad"]]
    return {"custom_ok": not bad_all, "reference_error": bool(ref_all),
            "why": "; ".join(bad_all + ref_all) or None}


def _gather_objects(obj, group):
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, obj, group=group)
    return out


def make_allreduce(group, device) -> AllReduce:
    return AllReduce(group, device)


def _is_gloo(group) -> bool:
    try:
        return dist.get_backend(group) == "gloo"
    except Exception:  # noqa: BLE001
        return False


def make_sp_collectives(group, device):
    """Sequence-parallel pair (SURVEY §2.3 "Megatron SP"): ``reduce_scatter(y)``
    sums the row-parallel partials ``y [tp*Tp, H]`` over the group and returns
    this rank's ``[Tp, H]`` row block; ``all_gather(x)`` concatenates every
    rank's ``[Tp, H]`` block into ``[tp*Tp, H]`` (rank order).  Together they
    move the same bytes as the all-reduce they replace (C1/C2), but the
    residual stream and the RMSNorms in between touch only ``Tp`` rows per rank.
    GPU: the direct RCCL communicator; CPU: gloo in fp32 (gloo has no
    reduce-scatter, so it is all-reduce + slice there).

    Each function carries ``graph_safe``: whether it can be captured in a
    hipGraph (RCCL on the capture stream is; gloo is host code and is not),
    which is what lets the engine capture sequence-parallel steps."""
    device = torch.device(device)
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    if device.type != "cuda":
        def cpu_rs(y: torch.Tensor) -> torch.Tensor:
            yf = y.float()
            dist.all_reduce(yf, group=group)
            tp_rows = y.shape[0] // world
            return yf[rank * tp_rows:(rank + 1) * tp_rows].to(y.dtype).contiguous()

        def cpu_ag(x: torch.Tensor) -> torch.Tensor:
            parts = [torch.empty_like(x, dtype=torch.float32) for _ in range(world)]
            dist.all_gather(parts, x.float().contiguous(), group=group)
            return torch.cat(parts).to(x.dtype)
        return _tag(cpu_rs, cpu_ag, safe=False)
    if os.environ.get("MCP_COMM", "native") == "native":
        comm = NativeComm(group, device)

        def gpu_rs(y: torch.Tensor) -> torch.Tensor:
            return comm.reduce_scatter(y).view(y.shape[0] // world, *y.shape[1:])

        def gpu_ag(x: torch.Tensor) -> torch.Tensor:
            return comm.all_gather(x).view(world * x.shape[0], *x.shape[1:])
        return _tag(gpu_rs, gpu_ag, safe=True)

    def torch_rs(y: torch.Tensor) -> torch.Tensor:
        out = y.new_empty(y.shape[0] // world, *y.shape[1:])
        dist.reduce_scatter_tensor(out, y.contiguous(), group=group)
        return out

    def torch_ag(x: torch.Tensor) -> torch.Tensor:
        out = x.new_empty(world * x.shape[0], *x.shape[1:])
        dist.all_gather_into_tensor(out, x.contiguous(), group=group)
        return out
    return _tag(torch_rs, torch_ag, safe=not _is_gloo(group))


def _tag(rs, ag, safe: bool):
    rs.graph_safe = ag.graph_safe = safe
    return rs, ag


class StepBroadcaster:
    """Driver -> worker step descriptors for tensor-parallel engines."""

    HDR = 32

    def __init__(self, group, device, src: int = 0):
        self.group, self.device, self.src = group, torch.device(device), src
        self._gloo = _is_gloo(group)

    def _bcast(self, t: torch.Tensor):
        if t.is_cuda and self._gloo:               # gloo moves host tensors only
            h = t.cpu()
            dist.broadcast(h, src=self.src, group=self.group)
            t.copy_(h)
            return
        dist.broadcast(t, src=self.src, group=self.group)

    def send(self, payload: torch.Tensor, layout) -> None:
        hdr = np.full(self.HDR, 0, np.int32)
        hdr[0], hdr[1] = payload.numel(), len(layout)
        hdr[2:2 + len(layout)] = layout
        self._bcast(torch.from_numpy(hdr).to(self.device))
        if payload.numel():
            self._bcast(payload if payload.device == self.device else payload.to(self.device))

    GRAPH = -2          # hdr[1] marker: replay the captured graph hdr[2:6]

    def send_graph(self, key, n: int) -> None:
        """Graph step: header (the graph key) first, so every worker can
        capture the same graph (its eager warm-up runs the same collectives)
        before the static payload is broadcast into the graph's buffer."""
        hdr = np.full(self.HDR, 0, np.int32)
        hdr[0], hdr[1] = n, self.GRAPH
        hdr[2:2 + len(key)] = key
        hdr[self.HDR - 1] = len(key)
        self._bcast(torch.from_numpy(hdr).to(self.device))

    def send_payload(self, payload: torch.Tensor) -> None:
        if payload.numel():
            self._bcast(payload)

    def stop(self) -> None:
        hdr = np.zeros(self.HDR, np.int32)
        hdr[0] = -1
        self._bcast(torch.from_numpy(hdr).to(self.device))

    def recv(self, graph_buffer=None):
        """Next message: None (stop), ``(payload, layout)`` (eager step) or,
        for a graph step, ``(buf, ("graph", key))`` after the payload landed in
        ``graph_buffer(key)`` (the worker's captured bucket buffer)."""
        hdr = torch.zeros(self.HDR, dtype=torch.int32, device=self.device)
        self._bcast(hdr)
        h = hdr.cpu().numpy()
        n, nl = int(h[0]), int(h[1])
        if n < 0:
            return None
        if nl == self.GRAPH:
            key = tuple(int(x) for x in h[2:2 + int(h[self.HDR - 1])])
            buf = graph_buffer(key)[:n]
            if n:
                self._bcast(buf)
            return buf, ("graph", key)
        layout = [int(x) for x in h[2:2 + nl]]
        payload = torch.empty(n, dtype=torch.int32, device=self.device)
        if n:
            self._bcast(payload)
        return payload, layout
