"""On-node planner: intent -> grammar-constrained Llama-3 decode -> T2 DAG.

This is the MI355X replacement of ``GraphPlanner.plan`` (control_plane.py:57-75):

1. list the registry (sorted, control_plane.py:58 / SURVEY D12);
2. if the registry is larger than ``retrieval_threshold``, keep the top-k
   services by cosine similarity between the intent and the HBM-resident
   schema embeddings (the never-called pgvector helper of
   control_plane.py:51-55, now a HIP top-k kernel, ``retrieval``);
3. build the prompt (shared registry prefix + per-intent suffix);
4. decode under the DAG grammar on the local engine at temperature 0.2
   (control_plane.py:72) - the output is valid T2 JSON by construction.

Concurrency: a dedicated scheduler thread owns the engine (and the GPU); the
asyncio side submits requests through a queue and awaits futures, so the
FastAPI event loop never blocks (fixes SURVEY D9).  ``plan_many`` is the
synchronous batch path used by the benchmark.
"""
from __future__ import annotations

import os

import asyncio
import queue
import threading
import time
from typing import Dict, List, Optional, Sequence

from ..utils.metrics import METRICS
from .base import Planner
from .grammar import GrammarSpec
from .prompt import build_prompt_parts
from .tokenizer import get_tokenizer, tokenizer_for


class EngineStalled(RuntimeError):
    """The engine made no progress for ``watchdog_s`` with requests pending
    (e.g. a hung GPU step); the API answers 503 and the router drains the replica.

    Recovery: the watchdog fails the pending requests at once; when the stuck
    step returns, the scheduler thread aborts everything the engine still
    holds (``LLMEngine.abort_all``) and clears ``stalled``, so new requests are
    served again.  A step that never returns needs a process restart (the DP
    router respawns its replicas; a lone server reports 503 on /healthz)."""


class LocalPlanner(Planner):
    def __init__(self, engine, registry, tokenizer=None, max_nodes: int = 6, retriever=None,
                 retrieval_threshold: int = 48, topk: int = 32, min_nodes: int = 1,
                 watchdog_s: Optional[float] = None):
        self.engine = engine
        self.registry = registry
        self.tok = tokenizer or get_tokenizer()
        self.max_nodes = max_nodes
        self.min_nodes = min_nodes
        self.retriever = retriever
        self.retrieval_threshold = retrieval_threshold
        self.topk = topk
        self._spec_cache: Dict[tuple, GrammarSpec] = {}
        self._prefix_cache: Dict[tuple, List[int]] = {}
        self._q: "queue.Queue" = queue.Queue()
        self._thread: Optional[threading.Thread] = None
        self._stop = threading.Event()
        self._lock = threading.Lock()
        self.watchdog_s = float(os.environ.get("MCP_WATCHDOG_S", "60")) if watchdog_s is None \
            else watchdog_s
        self._pending: Dict[int, tuple] = {}        # id -> (loop, future), async requests in flight
        self._pending_lock = threading.Lock()
        self._watchdog: Optional[threading.Thread] = None
        self.stalled = False
        # retrieval counts and their rank snapshot (MCP_RETRIEVAL_ORDER=popular)
        self._pop = {"counts": {}, "rank": {}, "n": 0, "lock": threading.Lock()}
        # MCP_PREP_THREAD (default 1): the per-request host phases (retrieval,
        # grammar, tokenisation) run on their own thread, so the engine thread
        # only schedules and launches steps; the prep thread's Python work
        # runs while the engine thread waits on the GPU (which releases the
        # GIL).  Config 3 (16 clients, 10k services): 45.8 vs 43.9 plans/s,
        # TTFT p99 192 vs 272 ms (profiles/config3_sched_sweep_r6.md)
        self.prep_thread = os.environ.get("MCP_PREP_THREAD", "1") == "1"
        self._prepq: "queue.Queue" = queue.Queue()
        self._prep: Optional[threading.Thread] = None

    # ----------------------------------------------------------- factory
    @classmethod
    def from_settings(cls, settings, registry):
        import torch
        from ..engine.engine import LLMEngine
        from ..models.llama import LlamaModel
        from ..retrieval.store import SchemaIndex
        from ..models.weights import model_from_checkpoint
        dev = "cuda:0" if torch.cuda.is_available() else "cpu"
        if os.path.isdir(settings.model):        # an HF safetensors checkpoint directory
            model = model_from_checkpoint(settings.model, dev)
        else:                                     # a named architecture, random-init weights
            model = LlamaModel.random(settings.model, dev, seed=settings.seed)
        kw = {} if dev != "cpu" else {"num_blocks": 512}
        if getattr(settings, "kv_blocks", 0):
            kw["num_blocks"] = settings.kv_blocks
        eng = LLMEngine(model, max_batch=settings.max_batch, max_step_tokens=settings.max_step_tokens,
                        temperature=settings.temperature, seed=settings.seed, **kw)
        if os.environ.get("MCP_GRAPH_WARM", "1") == "1":
            # capture the hipGraph buckets at start-up, not under the first requests
            eng.warm_graphs(max_tokens=settings.max_step_tokens)
        retr = SchemaIndex(registry, dim=settings.embed_dim, device=dev)
        retr.refresh()                     # embed the registry once, before serving
        retr.start_background()            # later registrations: incremental, off the engine thread
        tok = tokenizer_for(settings.model)
        if tok.vocab_size > model.cfg.vocab_size:
            raise ValueError(f"tokenizer vocabulary {tok.vocab_size} exceeds the model's "
                             f"{model.cfg.vocab_size}")
        planner = cls(eng, registry, tokenizer=tok, max_nodes=settings.max_nodes,
                      min_nodes=getattr(settings, "min_nodes", 1), retriever=retr,
                      retrieval_threshold=settings.retrieval_threshold, topk=settings.topk)
        # (no heap.settle() here: freezing the GC heap is a process entry
        # point's decision - the server's lifespan, a router replica, a bench)
        return planner

    # ----------------------------------------------------------- prepare
    # Retrieved services go into the prompt in a canonical order, so the
    # prompts of requests with overlapping retrieved sets share leading
    # 64-token blocks, which the engine's block-level prefix cache computes
    # once.  MCP_RETRIEVAL_ORDER:
    #   popular (default) - most often retrieved first (ties and unranked
    #     services by name): the services most requests retrieve form a common
    #     leading run and the rarely retrieved ones trail it, where a
    #     difference costs the fewest blocks.  The rank is a snapshot of the
    #     retrieval counts, re-taken at geometrically spaced request counts
    #     (16, 64, ... 16384, then every 16384), so the order - and the cached
    #     blocks - stay put between snapshots;
    #   name - name order; score - the similarity order.
    # Reproducibility: under "popular" the prompt of an intent depends on the
    # process's earlier traffic (the rank snapshot), so the same intent can
    # plan differently on another replica or later in the run.  Sampled plans
    # (temperature 0.2, control_plane.py:72) depend on that history anyway -
    # the Gumbel counter is (request uid, sample) - so for reproducible plans
    # run temperature 0 with MCP_RETRIEVAL_ORDER=name: the prompt is then a
    # function of the intent and the registry only.
    # 10k-service registry, 320 synthetic intents, top-32, a CPU replay of the
    # prompts' 64-token block chains: 69 % of the prefix blocks shared in
    # popularity order, 53 % in name order, 34 % in score order
    # (tests/test_planner_cpu.py replays a smaller registry).
    ORDER = os.environ.get("MCP_RETRIEVAL_ORDER", "popular")
    _RANK_AT = (16, 64, 256, 1024, 4096, 16384)

    def candidates(self, intent: str, services: Sequence[dict]) -> List[dict]:
        if self.retriever is None or len(services) <= self.retrieval_threshold:
            return list(services)
        found = self.retriever.search(intent, self.topk, services)
        if self.ORDER == "name":
            return sorted(found, key=lambda s: s["name"])
        if self.ORDER == "popular":
            return self._popular_order(found)
        return found

    def _popular_order(self, found: List[dict]) -> List[dict]:
        st = self._pop
        with st["lock"]:
            counts = st["counts"]
            for svc in found:
                nm = svc["name"]
                counts[nm] = counts.get(nm, 0) + 1
            st["n"] += 1
            n = st["n"]
            if n in self._RANK_AT or (n > self._RANK_AT[-1] and n % self._RANK_AT[-1] == 0):
                order = sorted(counts.items(), key=lambda kv: (-kv[1], kv[0]))
                st["rank"] = {nm: r for r, (nm, _) in enumerate(order)}
            rank = st["rank"]
        last = len(rank)
        return sorted(found, key=lambda svc: (rank.get(svc["name"], last), svc["name"]))

    def prepare(self, intent: str, services: Optional[Sequence[dict]] = None):
        """Per-request host phases: registry read + top-k
        retrieval (``retrieval_s``), grammar / prompt build + tokenisation
        (``prompt_s``); the engine adds queue / TTFT / decode / parse."""
        t0 = time.perf_counter()
        services = self.registry.list_services() if services is None else services
        dec, ptoks, t1 = self._decoder_and_prefix(intent, services, timed=True)
        stoks = self.tok.encode(self.suffix_text(intent))
        METRICS.observe("retrieval_s", t1 - t0)
        METRICS.observe("prompt_s", time.perf_counter() - t1)
        return dec, ptoks, stoks

    def _decoder_and_prefix(self, intent: str, services: Sequence[dict], timed: bool = False):
        cands = self.candidates(intent, services)
        t1 = time.perf_counter() if timed else None
        key = tuple(s["name"] for s in cands) + (getattr(self.registry, "version", 0),)
        spec = self._spec_cache.get(key)
        if spec is None:
            spec = GrammarSpec(cands, self.tok, max_nodes=self.max_nodes, min_nodes=self.min_nodes)
            if len(self._spec_cache) > 256:
                self._spec_cache.clear()
            self._spec_cache[key] = spec
        ptoks = self._prefix_cache.get(key)
        if ptoks is None:
            prefix, _ = build_prompt_parts(cands, intent, compact=spec.compact)
            ptoks = self.tok.prompt_ids(prefix)
            if len(self._prefix_cache) > 256:
                self._prefix_cache.clear()
            self._prefix_cache[key] = ptoks
        return (spec.decoder(), ptoks, t1) if timed else (spec.decoder(), ptoks)

    @staticmethod
    def suffix_text(intent: str) -> str:
        return f"\nUser intent: “{intent}”\n\nJSON DAG:"

    # ------------------------------------------------------- batch (sync)
    def submit_many(self, intents: Sequence[str], fresh_prefix: bool = True,
                    launch_ahead: bool = False) -> list:
        """Queue a batch of intents on the engine (the caller drives
        ``engine.step()``; ``plan_many`` = this + run).  ``launch_ahead``: the
        batch's shared registry-prefix job is created and launched on the GPU
        first, and the per-intent suffixes are tokenised while it runs (the
        caller must be the engine's only driver)."""
        services = self.registry.list_services()
        seqs = []
        batch_enc = getattr(self.tok, "encode_batch", None)
        if launch_ahead and intents and batch_enc and (self.retriever is None or
                                                       len(services) <= self.retrieval_threshold):
            _, ptoks0 = self._decoder_and_prefix(intents[0], services)
            if self.engine.get_prefix(ptoks0) is not None:
                self.engine.launch_ahead()
        sufs = batch_enc([self.suffix_text(it) for it in intents]) if batch_enc else None
        for i, it in enumerate(intents):
            if sufs is not None and (self.retriever is None or
                                     len(services) <= self.retrieval_threshold):
                dec, ptoks = self._decoder_and_prefix(it, services)
                stoks = sufs[i]
            else:
                dec, ptoks, stoks = self.prepare(it, services)
            seqs.append(self.engine.submit(dec, stoks, prefix_tokens=ptoks))
        if fresh_prefix:
            # batch-local prefix: this batch's requests hold their references,
            # the next batch recomputes it
            self.engine.drop_prefixes()
        return seqs

    def plan_many(self, intents: Sequence[str], fresh_prefix: bool = True) -> List[dict]:
        """Plan a batch of intents to completion on the calling thread."""
        with self._lock:
            seqs = self.submit_many(intents, fresh_prefix, launch_ahead=True)
            self.engine.run()
        out = []
        for s in seqs:
            if s.error:
                raise RuntimeError(s.error)
            out.append(s.result)
        return out

    # ------------------------------------------------------ async service
    def _ensure_thread(self):
        if self._thread is None or not self._thread.is_alive():
            self._thread = threading.Thread(target=self._loop, name="mcp-engine", daemon=True)
            self._thread.start()
        if self.prep_thread and (self._prep is None or not self._prep.is_alive()):
            self._prep = threading.Thread(target=self._prep_loop, name="mcp-prep", daemon=True)
            self._prep.start()
        if self.watchdog_s > 0 and (self._watchdog is None or not self._watchdog.is_alive()):
            self._watchdog = threading.Thread(target=self._watch, name="mcp-watchdog", daemon=True)
            self._watchdog.start()

    def _watch(self):
        """Fail every pending request if the engine stops making progress."""
        period = min(1.0, self.watchdog_s / 4)
        while not self._stop.wait(period):
            with self._pending_lock:
                busy = bool(self._pending)
            if not busy or self.stalled:
                continue
            idle = time.perf_counter() - self.engine.last_progress
            if idle > self.watchdog_s:
                self.stalled = True
                METRICS.inc("engine_stalls")
                with self._pending_lock:
                    items, self._pending = list(self._pending.values()), {}
                err = EngineStalled(f"planner engine made no progress for {idle:.1f}s")
                for loop, fut in items:
                    loop.call_soon_threadsafe(_set_exc, fut, err)

    def _submit_item(self, item):
        intent, loop, fut = item[:3]
        try:
            # prepared on the prep thread, or here
            dec, ptoks, stoks = item[3] if len(item) > 3 else self.prepare(intent)
            t0 = time.perf_counter()

            def done(seq, loop=loop, fut=fut, t0=t0):
                METRICS.observe("engine_latency_s", time.perf_counter() - t0)
                with self._pending_lock:
                    self._pending.pop(id(fut), None)
                if seq.error:
                    loop.call_soon_threadsafe(_set_exc, fut, RuntimeError(seq.error))
                else:
                    loop.call_soon_threadsafe(_set_result, fut, seq.result)
            self.engine.submit(dec, stoks, prefix_tokens=ptoks, on_done=done)
        except Exception as e:  # noqa: BLE001
            loop.call_soon_threadsafe(_set_exc, fut, e)

    def _pump(self) -> int:
        """Submit every request already queued (the engine's arrival pump,
        called on the engine thread while a lookahead launch is held)."""
        n = 0
        while True:
            try:
                item = self._q.get_nowait()
            except queue.Empty:
                return n
            self._submit_item(item)
            n += 1

    def _loop(self):
        eng = self.engine
        eng.poll_arrivals = self._pump
        while not self._stop.is_set():
            try:
                block = not eng.has_work()
                item = self._q.get(timeout=0.05) if block else self._q.get_nowait()
            except queue.Empty:
                item = None
            if item is not None:
                self._submit_item(item)
                self._pump()
            if eng.has_work():
                with self._lock:
                    eng.step()
            if self.stalled:                  # the stuck step returned: start over
                with self._lock:
                    n = eng.abort_all("planner engine stalled; request aborted")
                METRICS.inc("engine_recoveries")
                METRICS.inc("aborted_requests", n)
                self.stalled = False

    def _prep_loop(self):
        while not self._stop.is_set():
            try:
                intent, loop, fut = self._prepq.get(timeout=0.05)
            except queue.Empty:
                continue
            try:
                self._q.put((intent, loop, fut, self.prepare(intent)))
            except Exception as e:  # noqa: BLE001
                loop.call_soon_threadsafe(_set_exc, fut, e)

    async def plan(self, intent: str) -> dict:
        if self.stalled:
            raise EngineStalled("planner engine is stalled")
        self._ensure_thread()
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        with self._pending_lock:
            self._pending[id(fut)] = (loop, fut)
        (self._prepq if self.prep_thread else self._q).put((intent, loop, fut))
        return await fut

    async def aclose(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
        if self._prep is not None:
            self._prep.join(timeout=5)


def _set_result(fut, v):
    if not fut.done():
        fut.set_result(v)


def _set_exc(fut, e):
    if not fut.done():
        fut.set_exception(e)
