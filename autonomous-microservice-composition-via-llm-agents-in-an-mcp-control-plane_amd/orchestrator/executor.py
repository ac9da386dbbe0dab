"""DAG executor (CPU side).

Parity surface with the reference ``Orchestrator.execute``
(control_plane.py:87-131):

* graph construction: NetworkX ``DiGraph`` from ``graph["nodes"]`` (node attrs =
  the whole node dict) and ``graph["edges"]`` (edge attr ``fallback``)
  (:94-100).  A missing ``edges`` key, an edge to an unknown node and a cycle
  raise exactly like the reference (KeyError / KeyError('endpoint') /
  NetworkXUnfeasible -> HTTP 500), see SURVEY §2.4 T2.
* order: ``nx.topological_sort`` = generational Kahn order; ``results`` keys
  follow it (T3).
* inputs: ``{k: results.get(v, payload.get(v))}`` – the whole upstream JSON body
  or the payload field (T4).
* call: ``POST endpoint json=inputs timeout=5.0``, ``raise_for_status`` then
  ``.json()`` (T5); error strings are ``str(exception)`` verbatim (T6).
* fallback: the FIRST in-edge's ``fallback`` (:116-119).  The reference indexes
  the edge-attribute dict by node name (:119, always ``KeyError``);
  we implement the intended ``.get("fallback")``.
* no fallback -> ``HTTPException(502, "<name> failed and no fallback available")``
  (:130, T7), partial results discarded.
* log lines of logger ``orchestrator`` (:113, :121, :127, T9).

Extensions (all default to parity behaviour):

* per-node ``retries`` (README.md:49 claims per-node retry counts; the
  reference has none): node attr ``retries`` or ``Settings.retries``;
* ordered fallbacks: after the first-in-edge fallback, node-level ``fallback``
  / ``fallbacks`` and (opt-in) the registry record's ``fallback`` (T1);
* generation-level concurrency (opt-in): independent nodes of one topological
  generation run concurrently; ``results``/``errors`` keep topo order;
* telemetry: per-call latency/outcome to the metrics sink and (opt-in) to the
  registry (README.md:43-44).
"""
from __future__ import annotations

import asyncio
import json
import logging
import time
from typing import Any, Callable, Dict, List, Optional

import httpx
import networkx as nx
from fastapi import HTTPException

from ..utils.metrics import METRICS

logger = logging.getLogger("orchestrator")
_httpx_log = logging.getLogger("httpx")


class Orchestrator:
    def __init__(self, client: Optional[httpx.AsyncClient] = None, timeout: float = 5.0,
                 retries: int = 0, concurrent_generations: bool = False,
                 registry=None, use_registry_fallback: bool = False,
                 telemetry_to_registry: bool = False):
        self._own_client = client is None
        self.client = client if client is not None else httpx.AsyncClient()
        self.timeout = timeout
        self.retries = retries
        self.concurrent_generations = concurrent_generations
        self.registry = registry
        self.use_registry_fallback = use_registry_fallback
        self.telemetry_to_registry = telemetry_to_registry
        self.last_trace: List[Dict[str, Any]] = []

    async def aclose(self):
        if self._own_client:
            await self.client.aclose()

    # ------------------------------------------------------------ HTTP post
    # A service call is one POST of a JSON body.  ``client.post`` spends ~110 us
    # of Python per call in auth / redirect / cookie plumbing and URL merging
    # that an orchestrator call never uses (measured with a mock transport;
    # the reference pays it on every node, control_plane.py:109,123).  The fast
    # path builds the same request (client default headers, httpx's JSON
    # encoding, the per-request timeout), sends it on the client's own
    # transport for that URL (its connection pool, proxy mounts), and keeps
    # what the client would do with the response: the INFO line of logger
    # ``httpx``, cookie extraction, ``raise_for_status`` / ``.json()`` errors
    # with identical text (T5, T6).  Clients with auth, event hooks, cookies,
    # a base URL or redirect following take ``client.post``.
    def _fast_ok(self) -> bool:
        c = self.client
        ok = getattr(self, "_fast", None)
        # the client's default headers are re-read whenever they change (the
        # raw list is compared, not cached by identity): headers set on the
        # client after the first call are sent, as client.post would
        raw = c.headers.raw if isinstance(c, httpx.AsyncClient) else None
        if ok is None or ok[0] is not c or ok[4] != raw:
            usable = (isinstance(c, httpx.AsyncClient) and hasattr(c, "_transport_for_url")
                      and c.auth is None and not c.follow_redirects and not str(c.base_url)
                      and not any(c.event_hooks.values()) and not c.params)
            self._fast = ok = (c, usable, list(raw) if usable else None,
                               ok[3] if ok is not None and ok[0] is c else {}, raw)
        return ok[1] and not c.cookies

    async def _post(self, url: str, inputs: dict):
        if not self._fast_ok():
            resp = await self.client.post(url, json=inputs, timeout=self.timeout)
            resp.raise_for_status()
            return resp.json()
        c, _, base, urls, _ = self._fast
        if c.is_closed:                 # client.post's own check, same text
            raise RuntimeError("Cannot send a request, as the client has been closed.")
        u = urls.get(url)
        if u is None:
            if len(urls) > 4096:
                urls.clear()
            u = urls[url] = httpx.URL(url)
        body = json.dumps(inputs, ensure_ascii=False, separators=(",", ":"),
                          allow_nan=False).encode("utf-8")
        req = httpx.Request("POST", u, content=body, extensions={
            "timeout": httpx.Timeout(self.timeout).as_dict()},
            headers=base + [(b"Content-Length", str(len(body)).encode()),
                            (b"Content-Type", b"application/json")])
        resp = await c._transport_for_url(u).handle_async_request(req)
        resp.request = req
        try:
            await resp.aread()
        finally:
            await resp.aclose()
        if any(k.lower() == b"set-cookie" for k, _ in resp.headers.raw):
            c.cookies.extract_cookies(resp)
        resp.default_encoding = c._default_encoding
        _httpx_log.info('HTTP Request: %s %s "%s %d %s"', req.method, req.url, resp.http_version,
                        resp.status_code, resp.reason_phrase)
        resp.raise_for_status()
        return resp.json()

    # ------------------------------------------------------------------ graph
    @staticmethod
    def build_graph(graph: dict) -> nx.DiGraph:
        G = nx.DiGraph()
        for node in graph["nodes"]:
            G.add_node(node["name"], **node)
        for edge in graph["edges"]:
            G.add_edge(edge["from"], edge["to"], fallback=edge.get("fallback"))
        return G

    # ------------------------------------------------------------------- call
    async def _call(self, name: str, url: str, inputs: dict):
        t0 = time.perf_counter()
        ok = False
        try:
            out = await self._post(url, inputs)
            ok = True
            return out
        finally:
            dt = time.perf_counter() - t0
            METRICS.observe_service(name, dt, ok)
            self.last_trace.append({"node": name, "url": url, "ok": ok, "latency_s": dt})
            if self.telemetry_to_registry and self.registry is not None:
                try:
                    self.registry.record_call(name, dt, ok)
                except Exception:  # telemetry must never fail a request
                    pass

    def _fallbacks(self, G: nx.DiGraph, name: str, node: dict) -> List[str]:
        out: List[str] = []
        in_edges = list(G.in_edges(name))
        if in_edges:
            fb = G.edges[in_edges[0]].get("fallback")   # intended semantics of :119
            if fb:
                out.append(fb)
        extra = node.get("fallbacks")
        if isinstance(extra, list):
            out += [f for f in extra if isinstance(f, str) and f]
        if isinstance(node.get("fallback"), str) and node["fallback"]:
            out.append(node["fallback"])
        if self.use_registry_fallback and self.registry is not None:
            rec = self.registry.get(name)
            if rec is not None and rec.get("fallback"):
                out.append(rec["fallback"])
        seen, uniq = set(), []
        for f in out:
            if f not in seen:
                seen.add(f)
                uniq.append(f)
        return uniq

    async def _run_node(self, G: nx.DiGraph, name: str, payload: dict,
                        results: dict) -> tuple:
        """Returns (has_result, result, error_or_None).  May raise HTTPException(502)."""
        node = G.nodes[name]
        service_url = node["endpoint"]
        inputs = {k: results.get(v, payload.get(v)) for k, v in node["inputs"].items()}
        retries = node.get("retries", self.retries)
        retries = retries if isinstance(retries, int) and retries >= 0 else self.retries
        err: Optional[str] = None
        for attempt in range(retries + 1):
            try:
                return True, await self._call(name, service_url, inputs), err
            except Exception as e:
                logger.error(f"Service {name} failed: {e}")
                err = str(e)
                if attempt < retries:
                    logger.info(f"Retrying {name} ({attempt + 1}/{retries})")
        fallbacks = self._fallbacks(G, name, node)
        if not fallbacks:
            raise HTTPException(status_code=502, detail=f"{name} failed and no fallback available")
        for fb in fallbacks:
            logger.info(f"Attempting fallback {fb} for {name}")
            try:
                return True, await self._call(name, fb, inputs), err
            except Exception as e2:
                logger.error(f"Fallback {fb} failed: {e2}")
                err += f"; fallback failed: {e2}"
        return False, None, err

    # ---------------------------------------------------------------- execute
    async def execute(self, graph: dict, payload: dict) -> Dict[str, dict]:
        self.last_trace = []
        t0 = time.perf_counter()
        G = self.build_graph(graph)
        results: Dict[str, Any] = {}
        errors: Dict[str, str] = {}
        try:
            if not self.concurrent_generations:
                for name in nx.topological_sort(G):
                    ok, res, err = await self._run_node(G, name, payload, results)
                    if err is not None:
                        errors[name] = err
                    if ok:
                        results[name] = res
            else:
                await self._execute_generations(G, payload, results, errors)
        finally:
            METRICS.observe("execute_latency_s", time.perf_counter() - t0)
        return {"results": results, "errors": errors}

    @staticmethod
    def generations(G: nx.DiGraph) -> List[List[str]]:
        """Topological generations in networkx's generational-Kahn order (T3):
        the native runtime's ``topo_generations`` when built, else networkx.
        A cycle raises ``NetworkXUnfeasible`` either way (HTTP 500, as the
        reference's ``nx.topological_sort``)."""
        from ..engine import native
        if not native.available():
            return [list(g) for g in nx.topological_generations(G)]
        names = list(G.nodes)
        idx = {n: i for i, n in enumerate(names)}
        try:
            gens = native.topo_generations(len(names), [(idx[u], idx[v]) for u, v in G.edges])
        except RuntimeError as e:
            raise nx.NetworkXUnfeasible(str(e)) from None
        return [[names[i] for i in g] for g in gens]

    async def _execute_generations(self, G, payload, results, errors):
        gens = self.generations(G)
        order = [n for g in gens for n in g]
        pos = {n: i for i, n in enumerate(order)}
        gen_of: Dict[str, int] = {n: g for g, names in enumerate(gens) for n in names}
        i = 0
        while i < len(order):
            g = gen_of[order[i]]
            batch = [order[i]]
            j = i + 1
            # a node joins the concurrent batch unless it reads a result produced
            # by an earlier node of the same generation (serial semantics)
            while j < len(order) and gen_of[order[j]] == g:
                srcs = set(G.nodes[order[j]].get("inputs", {}).values()) \
                    if isinstance(G.nodes[order[j]].get("inputs"), dict) else set()
                if srcs & set(batch):
                    break
                batch.append(order[j])
                j += 1
            outs = await asyncio.gather(*[self._run_node(G, n, payload, results) for n in batch],
                                        return_exceptions=True)
            for n, o in sorted(zip(batch, outs), key=lambda t: pos[t[0]]):
                if isinstance(o, BaseException):
                    raise o
                ok, res, err = o
                if err is not None:
                    errors[n] = err
                if ok:
                    results[n] = res
            i = j
