"""Data-parallel planner replicas behind one API (SURVEY §2.3 "request-level DP",
§5.3 "the router drains a failed DP replica").

The reference is a single process with module singletons
(control_plane.py:135-138).  Here ``ReplicaRouter`` spawns one engine process
per GPU (``replicas`` of them, each a TP=1 Llama-3 replica pinned to its own
device, or a TP group launched separately), and implements the planner
interface:

* dispatch: least in-flight requests first (ties -> lowest index);
* results come back on one queue drained by a router thread that resolves the
  asyncio futures;
* failure handling: a replica whose process exits is marked dead and every
  request it had in flight is re-dispatched to a live replica; a request that
  exceeds ``request_timeout`` fails with TimeoutError (HTTP 500 at the API).

Queues carry only intent strings and DAG dicts produced by this process
tree.
"""
from __future__ import annotations

import asyncio
import itertools
import multiprocessing as mp
import os
import queue
import threading
import time
from typing import Dict, List, Optional

from ..planner.base import Planner


def _replica_main(idx: int, device: str, model: str, registry_records: list, inq, outq,
                  max_batch: int, max_nodes: int, seed: int, num_blocks: Optional[int]):
    """Replica process: owns one engine; plans batches of whatever is queued."""
    import torch
    from ..engine.engine import LLMEngine
    from ..models.llama import LlamaModel
    from ..registry import MemoryRegistry
    from .. planner.local import LocalPlanner
    if device.startswith("cuda"):
        torch.cuda.set_device(torch.device(device))
    m = LlamaModel.random(model, device, seed=seed)
    kw = {"num_blocks": num_blocks} if num_blocks else {}
    eng = LLMEngine(m, max_batch=max_batch, temperature=0.2, seed=seed + idx, **kw)
    planner = LocalPlanner(eng, MemoryRegistry(registry_records), max_nodes=max_nodes)
    outq.put(("ready", idx, None))
    pending = {}
    while True:
        try:
            item = inq.get(timeout=0.05 if eng.has_work() else 1.0)
        except queue.Empty:
            item = None
        while item is not None:
            if item == "stop":
                return
            rid, intent = item
            try:
                dec, ptoks, stoks = planner.prepare(intent)
                pending[rid] = eng.submit(dec, stoks, prefix_tokens=ptoks)
            except Exception as e:  # noqa: BLE001
                outq.put(("err", rid, repr(e)))
            try:
                item = inq.get_nowait()
            except queue.Empty:
                item = None
        if eng.has_work():
            eng.step()
        for rid in [r for r, s in pending.items() if s.done]:
            s = pending.pop(rid)
            outq.put(("err", rid, s.error) if s.error else ("ok", rid, s.result))


class ReplicaRouter(Planner):
    def __init__(self, devices: List[str], model: str, registry, max_batch: int = 256,
                 max_nodes: int = 6, seed: int = 0, num_blocks: Optional[int] = None,
                 request_timeout: float = 120.0, start_timeout: float = 600.0):
        self.registry = registry
        self.request_timeout = request_timeout
        ctx = mp.get_context("spawn")
        self._outq = ctx.Queue()
        self._inqs = []
        self._procs = []
        recs = [dict(s) for s in registry.list_services()]
        for i, dev in enumerate(devices):
            q = ctx.Queue()
            p = ctx.Process(target=_replica_main, daemon=True,
                            args=(i, dev, model, recs, q, self._outq, max_batch, max_nodes, seed,
                                  num_blocks))
            p.start()
            self._inqs.append(q)
            self._procs.append(p)
        self.alive = [True] * len(devices)
        self.inflight: Dict[int, Dict[int, str]] = {i: {} for i in range(len(devices))}
        self._futs: Dict[int, tuple] = {}
        self._ids = itertools.count()
        self._lock = threading.Lock()
        self._stop = threading.Event()
        ready, t0 = set(), time.time()
        while len(ready) < len(devices):
            if time.time() - t0 > start_timeout:
                raise TimeoutError("replicas did not start")
            try:
                kind, idx, _ = self._outq.get(timeout=1.0)
                if kind == "ready":
                    ready.add(idx)
            except queue.Empty:
                for i, p in enumerate(self._procs):
                    if not p.is_alive():
                        raise RuntimeError(f"replica {i} died during start-up")
        self._thread = threading.Thread(target=self._pump, daemon=True, name="mcp-router")
        self._thread.start()

    # -------------------------------------------------------------- routing
    def _pick(self) -> int:
        live = [i for i, a in enumerate(self.alive) if a]
        if not live:
            raise RuntimeError("no live planner replicas")
        return min(live, key=lambda i: (len(self.inflight[i]), i))

    def _dispatch(self, rid: int, intent: str):
        with self._lock:
            i = self._pick()
            self.inflight[i][rid] = intent
        self._inqs[i].put((rid, intent))

    def _pump(self):
        while not self._stop.is_set():
            try:
                kind, rid, val = self._outq.get(timeout=0.2)
            except queue.Empty:
                kind = None
            if kind in ("ok", "err"):
                with self._lock:
                    for d in self.inflight.values():
                        d.pop(rid, None)
                    entry = self._futs.pop(rid, None)
                if entry is not None:
                    loop, fut = entry
                    if kind == "ok":
                        loop.call_soon_threadsafe(_resolve, fut, val, None)
                    else:
                        loop.call_soon_threadsafe(_resolve, fut, None, RuntimeError(val))
            self._check_health()

    def _check_health(self):
        for i, p in enumerate(self._procs):
            if self.alive[i] and not p.is_alive():
                with self._lock:
                    self.alive[i] = False
                    orphans = list(self.inflight[i].items())
                    self.inflight[i].clear()
                for rid, intent in orphans:       # drain: re-dispatch to live replicas
                    try:
                        self._dispatch(rid, intent)
                    except RuntimeError as e:
                        entry = self._futs.pop(rid, None)
                        if entry:
                            entry[0].call_soon_threadsafe(_resolve, entry[1], None, e)

    async def plan(self, intent: str) -> dict:
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        rid = next(self._ids)
        self._futs[rid] = (loop, fut)
        self._dispatch(rid, intent)
        try:
            return await asyncio.wait_for(fut, self.request_timeout)
        finally:
            self._futs.pop(rid, None)

    def kill_replica(self, i: int):        # fault injection (tests)
        self._procs[i].kill()

    async def aclose(self):
        self._stop.set()
        for q, p in zip(self._inqs, self._procs):
            if p.is_alive():
                q.put("stop")
        for p in self._procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()


def _resolve(fut, val, exc):
    if fut.done():
        return
    if exc is not None:
        fut.set_exception(exc)
    else:
        fut.set_result(val)


def default_devices(n: int) -> List[str]:
    import torch
    if torch.cuda.is_available():
        return [f"cuda:{i}" for i in range(min(n, torch.cuda.device_count()))]
    return ["cpu"] * n
