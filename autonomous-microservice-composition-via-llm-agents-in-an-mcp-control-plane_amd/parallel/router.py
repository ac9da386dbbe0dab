"""Data-parallel planner replicas behind one API (SURVEY §2.3 "request-level DP",
§5.3 "the router drains a failed DP replica" / "restart the replica").

The reference is a single process with module singletons
(control_plane.py:135-138) that re-reads the Redis registry on every /plan
(control_plane.py:58 via :30-35).  Here ``ReplicaRouter`` spawns one engine
process per GPU (``replicas`` of them, each a TP=1 Llama-3 replica pinned to
its own device) and implements the planner interface:

* dispatch: least in-flight requests first (ties -> lowest index);
* registry freshness: a replica plans against the registry as it is when the
  request is dispatched.  With a Redis registry every replica opens its own
  ``RedisRegistry`` and re-reads it per request, exactly like the reference;
  with the in-memory registry the router compares ``registry.version`` at
  every dispatch and, when it changed, sends the new records down every
  replica's queue ahead of the request (queues are FIFO, so no request sees
  an older registry than the one current at its dispatch);
* retrieval-bounded prompts: every replica owns a ``SchemaIndex`` on its
  device (HBM-resident top-k cosine, the role of control_plane.py:51-55), so a
  registry larger than ``retrieval_threshold`` contributes only the ``topk``
  most similar services to the prompt;
* failure handling: a replica whose process exits, or that stops sending
  heartbeats for ``watchdog_s`` while it has requests in flight (a hung GPU
  step), is killed, every request it had in flight is re-dispatched to a live
  replica, and a fresh replica process is spawned in its place (at most
  ``max_respawns`` times per slot); a request that exceeds
  ``request_timeout`` fails with TimeoutError (HTTP 500 at the API).

Replicas of TP groups (``tp > 1``, e.g. 2 replicas of a TP=4 planner on one
8-GPU node): each replica is a group of ``tp`` processes with its own process
group on its own rendezvous port - the replica process is TP rank 0, the
driver (``LLMEngine(bcast=...)`` as in ``parallel.tp_serve``), and the router
spawns ranks 1..tp-1 as ``tp_serve`` workers next to it.  A group is one
failure unit: when any of its processes dies (or the driver stops sending
heartbeats with requests in flight - a rank lost mid-collective hangs the
others), every process of the group is killed and the group is respawned.

Queues carry only intent strings, registry records and DAG dicts produced by
this process tree.
"""
from __future__ import annotations

import asyncio
import dataclasses
import itertools
import multiprocessing as mp
import queue
import threading
import os
import time
from typing import Dict, List, Optional

from ..planner.base import Planner


@dataclasses.dataclass
class ReplicaConfig:
    model: str
    max_batch: int = 256
    max_nodes: int = 6
    min_nodes: int = 1
    seed: int = 0
    num_blocks: Optional[int] = None
    max_step_tokens: int = 8192
    temperature: float = 0.2
    retrieval_threshold: int = 48
    topk: int = 32
    embed_dim: int = 1024
    redis_url: Optional[str] = None     # replicas read Redis themselves when set
    services_prefix: Optional[str] = None
    heartbeat_s: float = 0.5
    tp: int = 1                         # ranks per replica (TP group size)
    tp_backend: Optional[str] = None    # default: nccl (RCCL) on GPUs, gloo on CPU
    full_weights_seed: Optional[int] = None   # tests: shard one full init (tp_serve.build_rank)
    # model == "stub": the replica answers every intent with this canned DAG
    # and runs no engine - measures the router / queue path alone
    stub_plan: Optional[dict] = None
    # stub replicas: each intent is answered this many seconds after it
    # reaches the replica (an engine's service time at any concurrency), and
    # optionally the whole replica stalls ``stub_stall_s`` once, ``stub_stall_at``
    # seconds after start-up (a hiccup such as a long GC pause or a slow step)
    stub_latency_s: float = 0.0
    stub_stall_at: float = -1.0
    stub_stall_s: float = 0.0


def _backend(cfg: ReplicaConfig, device: str) -> str:
    return cfg.tp_backend or ("nccl" if device.startswith("cuda") else "gloo")


class _Sender:
    """A replica's way back.  ``outq``: one router's queue, or - replicas
    shared by every API worker of a node (``SharedReplicas``) - a tuple
    (per-worker queues, supervisor queue): each result goes to the queue of
    the worker that dispatched it (request id mod workers), heartbeats to every
    worker and to the supervisor."""

    def __init__(self, idx: int, outq):
        self.idx = idx
        if isinstance(outq, tuple):
            self.workers, self.sup = list(outq[0]), outq[1]
        else:
            self.workers, self.sup = [outq], None

    def batch(self, items):
        if len(self.workers) == 1:
            self.workers[0].put(("batch", self.idx, items))
            return
        W = len(self.workers)
        by = {}
        for it in items:
            by.setdefault(it[1] % W, []).append(it)
        for w, its in by.items():
            self.workers[w].put(("batch", self.idx, its))

    def control(self, kind: str, val=None):
        for q in self.workers:
            q.put((kind, self.idx, val))
        if self.sup is not None:
            self.sup.put((kind, self.idx, val))


def _export_metrics(name: str):
    d = os.environ.get("MCP_METRICS_DIR")
    if d:
        from ..utils.metrics import METRICS
        METRICS.start_export(d, name)


def _replica_main(idx: int, device: str, cfg: ReplicaConfig, records: list, version: int,
                  inq, outq, port: Optional[int] = None):
    """Replica process: owns one engine; plans batches of whatever is queued.
    With ``cfg.tp > 1`` it is rank 0 (the driver) of its group's process
    group at ``port``; the router has spawned the other ranks."""
    out = _Sender(idx, outq)
    _export_metrics(f"replica-{idx}")
    if cfg.model == "stub":
        _stub_replica_main(idx, cfg, inq, out)
        return
    import torch
    from ..engine.engine import LLMEngine
    from ..models.llama import LlamaModel
    from ..planner.local import LocalPlanner
    from ..registry import MemoryRegistry, RedisRegistry
    from ..retrieval.store import SchemaIndex
    if device.startswith("cuda"):
        torch.cuda.set_device(torch.device(device))
    bcast = None
    if cfg.tp > 1:
        import torch.distributed as dist
        from .tp_serve import build_rank
        backend = _backend(cfg, device)
        kwd = {"device_id": torch.device(device)} if backend == "nccl" else {}
        dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=0,
                                world_size=cfg.tp, **kwd)
        m, nb, bcast = build_rank(cfg.model, 0, cfg.tp, device, cfg.seed, cfg.num_blocks,
                                  cfg.full_weights_seed)
        kw = {"num_blocks": nb}
    else:
        if os.path.isdir(cfg.model):                   # an HF checkpoint directory
            from ..models.weights import model_from_checkpoint
            m = model_from_checkpoint(cfg.model, device)
        elif cfg.full_weights_seed is not None:
            from ..models.llama import get_config, random_weights
            mc = get_config(cfg.model)
            m = LlamaModel(mc, random_weights(mc, device, seed=cfg.full_weights_seed), device)
        else:
            m = LlamaModel.random(cfg.model, device, seed=cfg.seed)
        kw = {"num_blocks": cfg.num_blocks} if cfg.num_blocks else {}
    eng = LLMEngine(m, max_batch=cfg.max_batch, max_step_tokens=cfg.max_step_tokens,
                    temperature=cfg.temperature, seed=cfg.seed + idx, bcast=bcast, **kw)
    if os.environ.get("MCP_GRAPH_WARM", "1") == "1":
        # capture the hipGraph buckets before reporting ready: the replica's
        # first requests replay instead of paying lazy captures
        eng.warm_graphs(max_tokens=cfg.max_step_tokens)
    if cfg.redis_url:
        registry = RedisRegistry(cfg.redis_url, **({"prefix": cfg.services_prefix}
                                                   if cfg.services_prefix else {}))
    else:
        registry = _VersionedMemoryRegistry(records, version)
    retriever = SchemaIndex(registry, dim=cfg.embed_dim, device=device)
    retriever.refresh()
    retriever.start_background()
    from ..utils.heap import settle as settle_heap
    settle_heap()                          # start-up heap -> permanent GC generation
    from ..planner.tokenizer import tokenizer_for
    planner = LocalPlanner(eng, registry, tokenizer=tokenizer_for(cfg.model),
                           max_nodes=cfg.max_nodes, min_nodes=cfg.min_nodes, retriever=retriever,
                           retrieval_threshold=cfg.retrieval_threshold, topk=cfg.topk)
    out.control("ready")
    pending = {}
    last_hb = time.monotonic()
    hb = _ReplicaWindow()
    while True:
        try:
            # never wait on the queue while the engine has a step to run
            item = inq.get_nowait() if eng.has_work() else inq.get(timeout=cfg.heartbeat_s)
        except queue.Empty:
            item = None
        while item is not None:
            if item == "stop":
                if bcast is not None:                  # release the worker ranks
                    import torch.distributed as dist
                    retriever.stop_background()
                    eng.shutdown_workers()
                    dist.destroy_process_group()
                return
            if item[0] == "registry":                  # ("registry", version, records)
                registry.replace(item[2], item[1])
            else:
                for rid, intent in (item[1] if item[0] == "many" else (item,)):
                    hb.received += 1
                    try:
                        dec, ptoks, stoks = planner.prepare(intent)
                        pending[rid] = eng.submit(dec, stoks, prefix_tokens=ptoks)
                    except Exception as e:  # noqa: BLE001
                        out.batch([("err", rid, repr(e))])
            try:
                item = inq.get_nowait()
            except queue.Empty:
                item = None
        if eng.has_work():
            t_step = time.perf_counter()
            eng.step()
            hb.step(time.perf_counter() - t_step)
        done = [r for r, s in pending.items() if s.done]
        if done:                                       # one message per step, not per request
            res = []
            for rid in done:
                s = pending.pop(rid)
                res.append(("err", rid, s.error) if s.error else ("ok", rid, s.result))
            hb.completed += len(res)
            out.batch(res)
        now = time.monotonic()
        if now - last_hb >= cfg.heartbeat_s:          # liveness for the router's watchdog
            out.control("hb", hb.snapshot(pending=len(pending), running=len(eng.running),
                                          waiting=len(eng.waiting)))
            last_hb = now


class _ReplicaWindow:
    """A replica's heartbeat payload: what it did since the last heartbeat
    (steps, step time, requests in / out, GC pauses) and its queue state now."""

    def __init__(self):
        from ..utils.procstats import GCWatch
        self.gc = GCWatch()
        self.t = time.monotonic()
        self.received = self.completed = self.steps = 0
        self.step_s = self.step_max_s = 0.0

    def step(self, dt: float):
        self.steps += 1
        self.step_s += dt
        self.step_max_s = max(self.step_max_s, dt)

    def snapshot(self, **now) -> dict:
        from ..utils.procstats import rss_mb
        t = time.monotonic()
        win = max(1e-9, t - self.t)
        out = {"window_s": round(win, 3), "received": self.received, "completed": self.completed,
               "steps": self.steps, "step_busy": round(self.step_s / win, 3),
               "step_max_ms": round(1e3 * self.step_max_s, 1), "rss_mb": round(rss_mb(), 1),
               "sent_at": time.time()}
        out.update(self.gc.snapshot())
        out.update(now)
        self.t = t
        self.received = self.completed = self.steps = 0
        self.step_s = self.step_max_s = 0.0
        return out


def _stub_replica_main(idx: int, cfg: ReplicaConfig, inq, sender: "_Sender"):
    """``model="stub"``: the replica's queue protocol with a canned planner
    (every intent gets ``cfg.stub_plan``), so tests and benches time the
    router, the queues and the API process alone.  With ``stub_latency_s``
    an intent is answered that long after it arrived, at any concurrency (an
    engine's service time), and ``stub_stall_at`` / ``stub_stall_s`` freeze
    the replica once (fault injection for the soak tests)."""
    import heapq
    plan = cfg.stub_plan or {"nodes": [], "edges": []}
    from ..utils.metrics import METRICS
    sender.control("ready")
    t_ready = last_hb = time.monotonic()
    delay = max(0.0, cfg.stub_latency_s)
    due: list = []                                     # (due time, seq, rid)
    seq = itertools.count()
    hb = _ReplicaWindow()
    stalled = cfg.stub_stall_at < 0
    while True:
        now = time.monotonic()
        if not stalled and now - t_ready >= cfg.stub_stall_at:
            stalled = True
            time.sleep(cfg.stub_stall_s)
            now = time.monotonic()
        wait = cfg.heartbeat_s if not due else max(0.0, min(cfg.heartbeat_s, due[0][0] - now))
        try:
            item = inq.get(timeout=wait) if wait > 0 else inq.get_nowait()
        except queue.Empty:
            item = None
        out = []
        while item is not None:
            if item == "stop":
                if out:
                    sender.batch(out)
                return
            if item[0] == "many":
                got = [rid for rid, _ in item[1]]
            elif item[0] != "registry":
                got = [item[0]]
            else:
                got = []
            hb.received += len(got)
            if delay > 0:
                t_due = time.monotonic() + delay
                for rid in got:
                    heapq.heappush(due, (t_due, next(seq), rid))
            else:
                out += [("ok", rid, plan) for rid in got]
            try:
                item = inq.get_nowait() if len(out) < 256 else None
            except queue.Empty:
                item = None
        now = time.monotonic()
        while due and due[0][0] <= now:
            out.append(("ok", heapq.heappop(due)[2], plan))
        if out:
            hb.completed += len(out)
            METRICS.plans_done(len(out), delay)       # the engine's own plan counter
            sender.batch(out)
        if now - last_hb >= cfg.heartbeat_s:
            sender.control("hb", hb.snapshot(pending=len(due), running=len(due), waiting=0))
            last_hb = now


class _VersionedMemoryRegistry:
    """The replica-side copy of an in-memory registry: the router's records
    and version, replaced wholesale when the router pushes a newer version."""

    def __init__(self, records, version: int):
        from ..registry import MemoryRegistry
        self._mk = MemoryRegistry
        self.replace(records, version)

    def replace(self, records, version: int):
        self._reg = self._mk(records)
        self._version = version

    @property
    def version(self) -> int:
        return self._version

    def list_services(self):
        return self._reg.list_services()

    def get(self, name):
        return self._reg.get(name)


def _spawn_group(ctx, i: int, cfg: ReplicaConfig, group: List[str], recs, version, inq, outspec):
    """Start replica ``i``: its TP worker ranks (``cfg.tp > 1``) and the
    replica process (rank 0) reading ``inq`` and answering to ``outspec``."""
    port = None
    workers = []
    if cfg.tp > 1:
        from .launch import free_port
        from .tp_serve import _worker_main
        port = free_port()
        env = {k: v for k, v in os.environ.items() if k.startswith(("MCP_", "HSA_"))}
        for r in range(1, cfg.tp):
            dev = group[r]
            w = ctx.Process(target=_worker_main, daemon=True,
                            args=(r, cfg.tp, port, dev, _backend(cfg, dev), cfg.model, cfg.seed,
                                  cfg.num_blocks, env, cfg.full_weights_seed))
            w.start()
            workers.append(w)
    p = ctx.Process(target=_replica_main, daemon=True,
                    args=(i, group[0], cfg, recs, version, inq, outspec, port))
    p.start()
    return p, workers


class ReplicaRouter(Planner):
    """``devices``: one device per replica (``tp = 1``), or one list of
    ``tp`` devices per replica (replicas of TP groups, ``group_devices``)."""

    def __init__(self, devices: List, model: str, registry, max_batch: int = 256,
                 max_nodes: int = 6, seed: int = 0, num_blocks: Optional[int] = None,
                 request_timeout: float = 120.0, start_timeout: float = 600.0,
                 watchdog_s: float = 60.0, max_respawns: int = 3,
                 config: Optional[ReplicaConfig] = None):
        self.registry = registry
        self.request_timeout = request_timeout
        self.start_timeout = start_timeout
        self.watchdog_s = watchdog_s
        self.max_respawns = max_respawns
        self.groups = [[d] if isinstance(d, str) else list(d) for d in devices]
        self.devices = [g[0] for g in self.groups]    # each replica's driver device
        cfg = config or ReplicaConfig(model=model, max_batch=max_batch, max_nodes=max_nodes,
                                      seed=seed, num_blocks=num_blocks,
                                      tp=len(self.groups[0]) if self.groups else 1)
        if any(len(g) != cfg.tp for g in self.groups):
            raise ValueError(f"every replica needs tp={cfg.tp} devices, got {self.groups}")
        from ..registry import RedisRegistry
        if isinstance(registry, RedisRegistry) and not cfg.redis_url:
            cfg = dataclasses.replace(cfg, redis_url=registry.client.url, services_prefix=registry.prefix)
        self.cfg = cfg
        self._ctx = mp.get_context("spawn")
        self._outq = self._ctx.Queue()
        n = len(devices)
        self._inqs: List = [None] * n
        self._procs: List = [None] * n
        self._workers: List[List] = [[] for _ in range(n)]   # TP ranks 1..tp-1 per replica
        self.alive = [False] * n
        self.respawns = [0] * n
        self._last_msg = [time.monotonic()] * n
        self.inflight: Dict[int, Dict[int, str]] = {i: {} for i in range(n)}
        self._futs: Dict[int, tuple] = {}
        self._ids = itertools.count()
        self._lock = threading.RLock()
        self._stop = threading.Event()
        self._pushed_version = None
        self._outbox: Dict[int, list] = {}          # replica -> requests awaiting the flush
        self._flush_scheduled = False
        self.replica_stats: List[Optional[dict]] = [None] * n   # last heartbeat payload
        self._win = {"dispatched": 0, "resolved": 0, "batches": 0, "transit_max_ms": 0.0}
        ensure_metrics_dir()              # replicas export their engine metrics for /metrics
        for i in range(n):
            self._spawn(i)
        t0 = time.time()
        while not all(self.alive):
            if time.time() - t0 > start_timeout:
                raise TimeoutError("replicas did not start")
            try:
                kind, idx, _ = self._outq.get(timeout=1.0)
                if kind == "ready":
                    self.alive[idx] = True
                    self._last_msg[idx] = time.monotonic()
            except queue.Empty:
                for i, p in enumerate(self._procs):
                    if not self._group_alive(i):
                        self._kill_group(i)
                        raise RuntimeError(f"replica {i} died during start-up")
        self._thread = threading.Thread(target=self._pump, daemon=True, name="mcp-router")
        self._thread.start()

    # ------------------------------------------------------------ replicas
    def _snapshot(self):
        """(version, records) of the in-memory registry (Redis replicas read it themselves)."""
        if self.cfg.redis_url:
            return 0, []
        return self.registry.version, [dict(s) for s in self.registry.list_services()]

    def _spawn(self, i: int):
        version, recs = self._snapshot()
        q = self._ctx.Queue()
        p, workers = _spawn_group(self._ctx, i, self.cfg, self.groups[i], recs, version, q,
                                  self._outq)
        self._inqs[i], self._procs[i], self._workers[i] = q, p, workers
        self._last_msg[i] = time.monotonic()

    def _group_alive(self, i: int) -> bool:
        p = self._procs[i]
        return p is not None and p.is_alive() and all(w.is_alive() for w in self._workers[i])

    def _kill_group(self, i: int):
        for proc in [self._procs[i]] + self._workers[i]:
            if proc is not None and proc.is_alive():
                proc.kill()
        for proc in [self._procs[i]] + self._workers[i]:
            if proc is not None:
                proc.join(timeout=10)

    # -------------------------------------------------------------- routing
    def _pick(self) -> int:
        live = [i for i, a in enumerate(self.alive) if a]
        if not live:
            raise RuntimeError("no live planner replicas")
        return min(live, key=lambda i: (len(self.inflight[i]), i))

    def _sync_registry(self):
        """Push the in-memory registry to every replica when its version moved."""
        if self.cfg.redis_url:
            return
        v = self.registry.version
        if v == self._pushed_version:
            return
        _, recs = self._snapshot()
        for i, q in enumerate(self._inqs):
            if q is not None:
                q.put(("registry", v, recs))
        self._pushed_version = v

    def _dispatch(self, rid: int, intent: str, loop=None):
        """Route one request to the least loaded live replica.  From the event
        loop (``loop`` given) the queue message is deferred to one flush per
        loop iteration and replica: a burst of requests crosses to each replica
        process as ONE message (one pickle, one pipe write, one feeder-thread
        wake-up) instead of one per request."""
        with self._lock:
            self._sync_registry()
            i = self._pick()
            self.inflight[i][rid] = intent
            self._assigned(i)
            self._win["dispatched"] += 1
            if loop is None:
                self._inqs[i].put((rid, intent))
                return
            pend = self._outbox.setdefault(i, [])
            pend.append((rid, intent))
            if not self._flush_scheduled:
                self._flush_scheduled = True
                loop.call_soon(self._flush)

    def _flush(self):
        with self._lock:
            box, self._outbox = self._outbox, {}
            self._flush_scheduled = False
            for i, items in box.items():
                q = self._inqs[i]
                if not self.alive[i] or q is None:
                    # the replica died since: the health check re-dispatches
                    # what it had in flight, these included
                    continue
                q.put(("many", items) if len(items) > 1 else items[0])

    def _pump(self):
        last_health = 0.0
        while not self._stop.is_set():
            try:
                kind, rid, val = self._outq.get(timeout=0.2)
            except queue.Empty:
                kind = None
            if kind in ("ready", "hb"):
                idx = rid
                with self._lock:
                    self._last_msg[idx] = time.monotonic()
                    if kind == "ready" and self._ready_ok(idx):
                        self.alive[idx] = True
                    elif kind == "hb" and val is not None:
                        # queue transit of the heartbeat: replica -> router lag
                        tr = 1e3 * (time.time() - val.get("sent_at", time.time()))
                        self._win["transit_max_ms"] = max(self._win["transit_max_ms"], tr)
                        self.replica_stats[idx] = val
            elif kind == "batch":                      # results of one replica step
                idx, done = rid, val
                resolve = []
                with self._lock:
                    self._last_msg[idx] = time.monotonic()
                    for k, r, v in done:
                        for i, d in self.inflight.items():
                            if d.pop(r, None) is not None:
                                self._released(i)
                                break
                        entry = self._futs.pop(r, None)
                        if entry is not None:
                            resolve.append((entry, k, v))
                    self._win["resolved"] += len(resolve)
                    self._win["batches"] += 1
                by_loop = {}
                for (loop, fut), k, v in resolve:
                    by_loop.setdefault(loop, []).append(
                        (fut, v, None) if k == "ok" else (fut, None, RuntimeError(v)))
                for loop, items in by_loop.items():     # one wake-up per event loop
                    loop.call_soon_threadsafe(_resolve_many, items)
            # liveness (process table syscalls) at most every 50 ms, not per message
            now = time.monotonic()
            if kind is None or now - last_health >= 0.05:
                last_health = now
                self._check_health()

    def _check_health(self):
        now = time.monotonic()
        for i, p in enumerate(self._procs):
            if p is None:
                continue
            dead = not self._group_alive(i)
            hung = (not dead and self.alive[i] and self.inflight[i]
                    and now - self._last_msg[i] > self.watchdog_s)
            if not dead and not hung:
                continue
            # a dead rank leaves the rest of its group blocked in a collective,
            # a stalled step leaves the whole group hung: replace every process
            self._kill_group(i)
            was_live = self.alive[i]
            with self._lock:
                self.alive[i] = False
                orphans = list(self.inflight[i].items())
                self.inflight[i].clear()
            if not was_live and not orphans and self._procs[i] is not p:
                continue
            for rid, intent in orphans:       # drain: re-dispatch to live replicas
                try:
                    self._dispatch(rid, intent)
                except RuntimeError as e:
                    entry = self._futs.pop(rid, None)
                    if entry:
                        entry[0].call_soon_threadsafe(_resolve, entry[1], None, e)
            if self.respawns[i] < self.max_respawns and not self._stop.is_set():
                self.respawns[i] += 1
                self._spawn(i)                # 'ready' marks it live again
            else:
                self._procs[i] = None

    def _ready_ok(self, idx: int) -> bool:
        return self._procs[idx] is not None and self._procs[idx].is_alive()

    # per-replica load hooks (SharedRouter keeps a node-wide count)
    def _assigned(self, i: int):
        pass

    def _released(self, i: int):
        pass

    def _next_rid(self) -> int:
        return next(self._ids)

    async def plan(self, intent: str) -> dict:
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        rid = self._next_rid()
        self._futs[rid] = (loop, fut)
        self._dispatch(rid, intent, loop)
        # a timer on the future instead of asyncio.wait_for (which wraps every
        # request in an extra task: ~20 % of the API process's time per plan
        # at thousands of plans/s)
        timer = loop.call_later(self.request_timeout, _resolve, fut, None,
                                TimeoutError(f"plan not done in {self.request_timeout:.0f}s"))
        try:
            return await fut
        finally:
            timer.cancel()
            self._futs.pop(rid, None)

    def stats(self) -> dict:
        """The router's window since the last call plus every replica's last
        heartbeat (``MCP_STATS_S`` lines of the API process)."""
        def qsize(q):
            try:
                return q.qsize()
            except (NotImplementedError, OSError, AttributeError):
                return -1
        with self._lock:
            win, self._win = self._win, {"dispatched": 0, "resolved": 0, "batches": 0,
                                         "transit_max_ms": 0.0}
            out = dict(win, transit_max_ms=round(win["transit_max_ms"], 1),
                       futures=len(self._futs),
                       inflight=[len(self.inflight[i]) for i in range(len(self._procs))],
                       alive=[bool(a) for a in self.alive], respawns=list(self.respawns),
                       outq=qsize(self._outq), inq=[qsize(q) if q is not None else -1
                                                    for q in self._inqs])
            out["replicas"] = [None if r is None else {k: v for k, v in r.items() if k != "sent_at"}
                               for r in self.replica_stats]
        return out

    def kill_replica(self, i: int):        # fault injection (tests)
        self._procs[i].kill()

    async def aclose(self):
        self.close()

    def close(self):
        self._stop.set()
        for q, p in zip(self._inqs, self._procs):
            if p is not None and p.is_alive():
                q.put("stop")
        for i, p in enumerate(self._procs):
            for proc in ([p] if p is not None else []) + self._workers[i]:
                proc.join(timeout=30)
                if proc.is_alive():
                    proc.kill()


def _resolve_many(items):
    for fut, val, exc in items:
        _resolve(fut, val, exc)


def _resolve(fut, val, exc):
    if fut.done():
        return
    if exc is not None:
        fut.set_exception(exc)
    else:
        fut.set_result(val)


def ensure_metrics_dir() -> str:
    """``MCP_METRICS_DIR`` for this process tree (created once, inherited by
    spawned children): every process exports its metrics there, and /metrics
    renders the node (utils/metrics.py)."""
    d = os.environ.get("MCP_METRICS_DIR")
    if not d:
        import tempfile
        base = "/dev/shm" if os.path.isdir("/dev/shm") else None
        d = tempfile.mkdtemp(prefix="mcp-metrics-", dir=base)
        os.environ["MCP_METRICS_DIR"] = d
        import atexit
        import shutil
        creator = os.getpid()
        # the creating process removes it (spawned children inherit the path only)
        atexit.register(lambda: os.getpid() == creator and shutil.rmtree(d, ignore_errors=True))
    return d


class SharedReplicas:
    """The node's replicas, shared by every API worker (VERDICT r5 missing
    #2: request-level balancing across workers).

    Round 5 gave each API worker a static slice of the replicas, so the
    kernel's SO_REUSEPORT hash - which spreads *connections*, not requests -
    decided which replicas worked: a client with two keep-alive connections
    kept two workers' slices busy and left the rest idle.  Here the API
    supervisor (which never initialises HIP) owns the replica processes and
    hands every worker the same handles:

    * one request queue per replica (any worker may dispatch to any replica);
    * one result queue per worker; a replica returns each result to the queue
      of the worker that sent it (request id mod workers, ``_Sender``);
    * ``load``: a shared [workers x replicas] table of requests in flight.
      Each worker writes only its own row, so no lock is needed; dispatch
      picks the live replica with the smallest column sum - least loaded
      across the whole node, whichever worker took the connection;
    * ``alive`` / ``epoch`` per replica: the supervisor watches the replica
      processes (exit, or no heartbeat for ``watchdog_s`` with work in
      flight), kills and respawns them and bumps the epoch; every worker that
      sees an epoch move re-dispatches what it had in flight there.

    The handle is pickled into each API worker process at spawn."""

    def __init__(self, groups: List, cfg: ReplicaConfig, registry, workers: int,
                 watchdog_s: float = 60.0, max_respawns: int = 3):
        self.ctx = mp.get_context("spawn")
        self.groups = [[d] if isinstance(d, str) else list(d) for d in groups]
        self.cfg = cfg
        self.W, self.R = workers, len(self.groups)
        self.inqs = [self.ctx.Queue() for _ in range(self.R)]
        self.outqs = [self.ctx.Queue() for _ in range(self.W)]
        self.supq = self.ctx.Queue()
        self.load = self.ctx.RawArray("l", self.W * self.R)
        self.alive = self.ctx.RawArray("b", self.R)
        self.epoch = self.ctx.RawArray("l", self.R)
        self.watchdog_s = watchdog_s
        self.max_respawns = max_respawns
        self._registry = registry
        self._procs = [None] * self.R
        self._workers: List[List] = [[] for _ in range(self.R)]
        self._last_msg = [time.monotonic()] * self.R
        self.respawns = [0] * self.R
        self._stop = None
        self.version0 = None

    def __getstate__(self):                 # what an API worker needs
        d = dict(self.__dict__)
        for k in ("_registry", "_procs", "_workers", "_stop", "_thread"):
            d.pop(k, None)
        d.pop("ctx", None)
        return d

    def __setstate__(self, d):
        self.__dict__.update(d)
        self.ctx = mp.get_context("spawn")

    # ------------------------------------------------- supervisor side
    def _snapshot(self):
        if self.cfg.redis_url or self._registry is None:
            return 0, []
        return self._registry.version, [dict(s) for s in self._registry.list_services()]

    def _spawn(self, i: int):
        version, recs = self._snapshot()
        p, ws = _spawn_group(self.ctx, i, self.cfg, self.groups[i], recs, version, self.inqs[i],
                             (self.outqs, self.supq))
        self._procs[i], self._workers[i] = p, ws
        self._last_msg[i] = time.monotonic()

    def _group_alive(self, i: int) -> bool:
        p = self._procs[i]
        return p is not None and p.is_alive() and all(w.is_alive() for w in self._workers[i])

    def _kill(self, i: int):
        for proc in [self._procs[i]] + self._workers[i]:
            if proc is not None and proc.is_alive():
                proc.kill()
        for proc in [self._procs[i]] + self._workers[i]:
            if proc is not None:
                proc.join(timeout=10)

    def inflight(self, i: int) -> int:
        return sum(self.load[w * self.R + i] for w in range(self.W))

    def start(self, start_timeout: float = 600.0):
        """Spawn every replica and wait until all are ready, then watch them
        from a supervisor thread."""
        ensure_metrics_dir()
        self.version0 = self._snapshot()[0] if not self.cfg.redis_url else None
        for i in range(self.R):
            self._spawn(i)
        t0 = time.time()
        while not all(self.alive):
            if time.time() - t0 > start_timeout:
                raise TimeoutError("replicas did not start")
            try:
                kind, idx, _ = self.supq.get(timeout=1.0)
                if kind == "ready":
                    self.alive[idx] = 1
                    self._last_msg[idx] = time.monotonic()
            except queue.Empty:
                for i in range(self.R):
                    if not self._group_alive(i):
                        self.close()
                        raise RuntimeError(f"replica {i} died during start-up")
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._watch, daemon=True, name="mcp-replicas")
        self._thread.start()

    def _watch(self):
        while not self._stop.is_set():
            try:
                kind, idx, _ = self.supq.get(timeout=0.2)
                self._last_msg[idx] = time.monotonic()
                if kind == "ready" and self._procs[idx] is not None:
                    self.alive[idx] = 1
            except queue.Empty:
                pass
            now = time.monotonic()
            for i in range(self.R):
                if self._procs[i] is None:
                    continue
                dead = not self._group_alive(i)
                hung = (not dead and self.alive[i] and self.inflight(i) > 0
                        and now - self._last_msg[i] > self.watchdog_s)
                if not dead and not hung:
                    continue
                self.alive[i] = 0
                self._kill(i)
                self.epoch[i] += 1              # workers re-dispatch what they had there
                if self.respawns[i] < self.max_respawns and not self._stop.is_set():
                    self.respawns[i] += 1
                    self._spawn(i)
                else:
                    self._procs[i] = None

    def kill_replica(self, i: int):          # fault injection (tests)
        self._procs[i].kill()

    def reset_worker(self, w: int):
        """An API worker died: its in-flight requests died with it."""
        for i in range(self.R):
            self.load[w * self.R + i] = 0

    def close(self):
        if self._stop is not None:
            self._stop.set()
        for i, q in enumerate(self.inqs):
            if self._procs[i] is not None and self._procs[i].is_alive():
                q.put("stop")
        for i, p in enumerate(self._procs):
            for proc in ([p] if p is not None else []) + self._workers[i]:
                proc.join(timeout=30)
                if proc.is_alive():
                    proc.kill()


class SharedRouter(ReplicaRouter):
    """One API worker's router over ``SharedReplicas``: dispatches to the
    node-wide least loaded live replica; spawns nothing (the supervisor owns
    the replica processes)."""

    def __init__(self, shared: SharedReplicas, worker: int, registry,
                 request_timeout: float = 120.0):
        self.shared = shared
        self.w = worker
        self.registry = registry
        self.request_timeout = request_timeout
        self.cfg = shared.cfg
        R = shared.R
        self._inqs = shared.inqs
        self._outq = shared.outqs[worker]
        self._procs = [None] * R
        self._workers = [[] for _ in range(R)]
        self.respawns = [0] * R
        self._last_msg = [time.monotonic()] * R
        self.inflight = {i: {} for i in range(R)}
        self._futs = {}
        self._ids = itertools.count()
        self._lock = threading.RLock()
        self._stop = threading.Event()
        # the replicas started on the supervisor's registry snapshot: push
        # only a newer version
        self._pushed_version = shared.version0
        self._outbox = {}
        self._flush_scheduled = False
        self.replica_stats = [None] * R
        self._win = {"dispatched": 0, "resolved": 0, "batches": 0, "transit_max_ms": 0.0}
        self._epochs = list(shared.epoch)
        self._row = worker * R
        self._cursor = worker * R // max(1, shared.W) - 1   # workers start apart
        d = os.environ.get("MCP_METRICS_DIR")
        if d:
            from ..utils.metrics import METRICS
            METRICS.start_export(d, f"api-{worker}")
        self._thread = threading.Thread(target=self._pump, daemon=True, name="mcp-router")
        self._thread.start()

    @property
    def alive(self):
        return self.shared.alive

    def _ready_ok(self, idx: int) -> bool:
        return False                        # the supervisor marks replicas live

    # A worker's home replicas (i % W == w) win unless some other replica has
    # more than HOME_SLACK fewer requests in flight node-wide.  Without the
    # preference every worker spread each burst over every replica, so each
    # replica split every result batch W ways and the queues carried W times
    # the messages: 4 workers x 8 stub replicas went from 20.8-23.3k to
    # 8.6-9.5k requests/s (tools/frontend_sweep.py, round 6).  Under skew
    # (a client on few connections) the home replicas fill and the rest take
    # the overflow.
    HOME_SLACK = int(os.environ.get("MCP_SHARED_HOME_SLACK", "1"))

    def _pick(self) -> int:
        """The live replica with the fewest requests in flight node-wide,
        this worker's home replicas first (``HOME_SLACK``); ties go
        round-robin from the last pick."""
        sh, R, W = self.shared, self.shared.R, self.shared.W
        load = sh.load[:]                      # one copy of the table (ctypes reads are slow)
        alive = sh.alive[:]
        best, best_v = -1, None
        home, home_v = -1, None
        start = self._cursor + 1
        for k in range(R):
            i = (start + k) % R
            if not alive[i]:
                continue
            v = sum(load[i::R])
            if best_v is None or v < best_v:
                best, best_v = i, v
            if i % W == self.w and (home_v is None or v < home_v):
                home, home_v = i, v
        if best < 0:
            raise RuntimeError("no live planner replicas")
        if home >= 0 and home_v <= best_v + self.HOME_SLACK:
            best = home
        self._cursor = best
        return best

    def _assigned(self, i: int):
        self.shared.load[self._row + i] += 1

    def _released(self, i: int):
        self.shared.load[self._row + i] -= 1

    def _next_rid(self) -> int:
        return next(self._ids) * self.shared.W + self.w

    def _check_health(self):
        """Re-dispatch what this worker had on a replica whose epoch moved
        (the supervisor killed / respawned it)."""
        for i in range(self.shared.R):
            e = self.shared.epoch[i]
            if e == self._epochs[i]:
                continue
            self._epochs[i] = e
            with self._lock:
                orphans = list(self.inflight[i].items())
                self.inflight[i].clear()
                self.shared.load[self._row + i] = 0
            for rid, intent in orphans:
                try:
                    self._dispatch(rid, intent)
                except RuntimeError as err:
                    entry = self._futs.pop(rid, None)
                    if entry:
                        entry[0].call_soon_threadsafe(_resolve, entry[1], None, err)

    def kill_replica(self, i: int):
        raise RuntimeError("replicas belong to the API supervisor (SharedReplicas.kill_replica)")

    def close(self):
        self._stop.set()


def default_devices(n: int) -> List[str]:
    """One device per replica: cuda:0 .. cuda:n-1 (as many as exist).
    ``MCP_REPLICA_DEVICES`` ("cuda:0,cuda:0", ...) places them explicitly -
    e.g. several replicas sharing one GPU for a one-GPU test of the
    multi-replica paths (size their KV pools with MCP_KV_BLOCKS then)."""
    forced = os.environ.get("MCP_REPLICA_DEVICES")
    if forced:
        devs = [d.strip() for d in forced.split(",") if d.strip()]
        return (devs * n)[:n]
    import torch
    if torch.cuda.is_available():
        return [f"cuda:{i}" for i in range(min(n, torch.cuda.device_count()))]
    return ["cpu"] * n


def group_devices(replicas: int, tp: int) -> List:
    """Device groups for ``replicas`` TP groups of ``tp`` ranks: replica i
    takes GPUs i*tp .. i*tp+tp-1 (contiguous, so a TP=4 group sits on one
    xGMI-adjacent half of the node); plain device strings when tp == 1.
    Counting devices does not initialise HIP, so the router can still spawn
    its children afterwards."""
    import torch
    if tp <= 1:
        return default_devices(replicas)
    n = torch.cuda.device_count()
    if n == 0:
        return [["cpu"] * tp for _ in range(replicas)]
    if replicas * tp > n:
        raise RuntimeError(f"{replicas} replicas x TP={tp} need {replicas * tp} GPUs, found {n}")
    return [[f"cuda:{i * tp + r}" for r in range(tp)] for i in range(replicas)]
