"""Planner backends.

Reference: ``GraphPlanner.plan`` (control_plane.py:57-75) lists the registry,
builds the prompt, calls OpenAI ``gpt-4o-mini`` at temperature 0.2 and
``json.loads`` the reply.  Here a planner is anything with
``async plan(intent) -> dict``:

* ``StubPlanner``   – canned JSON (BASELINE config 1: CPU plumbing, no GPU) or a
  deterministic keyword planner over the registry;
* ``LocalPlanner``  – the on-node Llama-3 engine with grammar-constrained
  decoding (``planner.local``).

Planning runs off the event loop (the reference blocks the loop in
``/plan_and_execute``, control_plane.py:149-150).
"""
from __future__ import annotations

import json
import re
import time
from typing import Optional

from ..utils.metrics import METRICS
from .prompt import PromptCache


class Planner:
    async def plan(self, intent: str) -> dict:
        raise NotImplementedError

    async def aclose(self):
        pass


class StubPlanner(Planner):
    """Canned-JSON planner.

    ``canned`` may be a dict (returned as-is), a str (``json.loads``-ed each
    call, so invalid text yields the reference's HTTP 500), or None: then a
    deterministic plan is derived from keyword overlap between the intent and
    the registry's service names.
    """

    def __init__(self, registry=None, canned=None, max_nodes: int = 4):
        self.registry = registry
        self.canned = canned
        self.max_nodes = max_nodes
        self.last_prompt: Optional[str] = None
        self._prompts = PromptCache()

    async def plan(self, intent: str) -> dict:
        t0 = time.perf_counter()
        services = self.registry.list_services() if self.registry is not None else []
        prefix, suffix = self._prompts.parts(services, intent, getattr(self.registry, "version", None))
        self.last_prompt = prefix + suffix
        if isinstance(self.canned, str):
            dag = json.loads(self.canned)
        elif self.canned is not None:
            dag = json.loads(json.dumps(self.canned))
        else:
            dag = self._keyword_plan(intent, services)
        METRICS.plan_done(time.perf_counter() - t0)
        return dag

    def _keyword_plan(self, intent, services) -> dict:
        words = set(re.findall(r"[a-z]+", intent.lower()))
        scored = []
        for i, s in enumerate(services):
            parts = set(s["name"].split("-"))
            scored.append((-len(parts & words), i, s))
        scored.sort(key=lambda t: (t[0], t[1]))
        chosen = [s for sc, _, s in scored[: self.max_nodes] if sc < 0] or [t[2] for t in scored[:1]]
        nodes, edges, prev = [], [], None
        for s in chosen:
            keys = s.input_keys() if hasattr(s, "input_keys") else []
            inputs = {k: (prev if (prev is not None and j == 0) else k) for j, k in enumerate(keys)}
            nodes.append({"name": s["name"], "endpoint": s["endpoint"], "inputs": inputs})
            if prev is not None:
                e = {"from": prev, "to": s["name"]}
                if s.get("fallback"):
                    e["fallback"] = s["fallback"]
                edges.append(e)
            prev = s["name"]
        return {"nodes": nodes, "edges": edges}


class CachedPlanner(Planner):
    """LRU plan cache keyed by (intent, registry version) in front of any
    planner (optional; ``MCP_PLAN_CACHE=<entries>``).  A registry
    change bumps its version and so misses every old entry.  Plans are
    returned as copies, so callers may mutate them."""

    def __init__(self, inner: Planner, registry=None, size: int = 1024):
        from collections import OrderedDict
        self.inner = inner
        self.registry = registry
        self.size = max(1, size)
        self._lru = OrderedDict()
        self.hits = self.misses = 0

    async def plan(self, intent: str) -> dict:
        key = (intent, getattr(self.registry, "version", None))
        dag = self._lru.get(key)
        if dag is not None:
            self._lru.move_to_end(key)
            self.hits += 1
            METRICS.inc("plan_cache_hits")
            return json.loads(dag)
        self.misses += 1
        out = await self.inner.plan(intent)
        self._lru[key] = json.dumps(out)
        if len(self._lru) > self.size:
            self._lru.popitem(last=False)
        return out

    async def aclose(self):
        await self.inner.aclose()

    def __getattr__(self, name):          # stalled / engine / ... of the wrapped planner
        return getattr(self.inner, name)

