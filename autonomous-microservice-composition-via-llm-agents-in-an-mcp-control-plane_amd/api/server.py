"""FastAPI surface.

Same routes and request/response field names as the reference
(control_plane.py:39-43, 79-85, 140-151):

* ``POST /plan``             {intent} -> {graph}
* ``POST /execute``          {graph, payload} -> {results, errors}
* ``POST /plan_and_execute`` {intent} -> {results, errors}  (payload ``{}``,
  control_plane.py:151)

plus ``GET /metrics`` (Prometheus text, README.md:43-44), ``GET /healthz`` and
the audit surface the reference README claims (README.md:50): ``POST /plan``
with ``"explain": true`` adds an ``explanation`` string next to ``graph`` (the
response is unchanged otherwise), and ``POST /explain`` {graph} ->
{explanation} (``planner/audit.py``).  ``MCP_ADAPTIVE=1`` hardens plans from
recorded service telemetry (README.md:43-44,48).

Differences by design: the app is built by a factory (no import-time DB
connection), the HTTP client is lifespan-managed (D14) and the
planner is awaited instead of blocking the event loop (D9).  Error semantics
are kept: a planner reply that is not a JSON object -> 500, missing
``intent`` -> 422, a failed node without fallback -> 502 (T7, T8).
"""
from __future__ import annotations

import contextlib
import logging
import os
from typing import Optional

import httpx
from fastapi import FastAPI, HTTPException
from fastapi.responses import JSONResponse, PlainTextResponse, Response
from pydantic import BaseModel

from ..config import Settings
from ..orchestrator import Orchestrator
from ..planner.base import Planner, StubPlanner
from ..registry import BaseRegistry, make_registry
from ..utils.metrics import METRICS

logging.basicConfig(level=logging.INFO)


class PlanRequest(BaseModel):
    intent: str
    explain: bool = False


class ExplainRequest(BaseModel):
    graph: dict


class ExplainResponse(BaseModel):
    explanation: str


class PlanResponse(BaseModel):
    graph: dict


class ExecuteRequest(BaseModel):
    graph: dict
    payload: dict


class ExecuteResponse(BaseModel):
    results: dict
    errors: dict


def plan_response_json(graph) -> bytes:
    """The ``/plan`` response body: the validated model serialised once (a
    non-object plan raises here -> 500, T8).  Shared by the FastAPI route and
    the fast front end (api/fasthttp.py)."""
    resp = PlanResponse(graph=graph)
    return resp.__pydantic_serializer__.to_json(resp)


def replica_slice(groups: list, spec: Optional[str]) -> list:
    """This API worker's share of the node's replicas: ``spec`` = "w/n" takes
    the contiguous groups [w R / n, (w + 1) R / n) of R (``None``: all)."""
    if not spec:
        return groups
    w, n = (int(x) for x in spec.split("/"))
    R = len(groups)
    if not 0 <= w < n <= R:
        raise ValueError(f"replica slice {spec} of {R} replicas")
    return groups[w * R // n:(w + 1) * R // n]


def _stub_plan(registry: BaseRegistry, settings: Settings) -> Optional[dict]:
    """Stub replicas' canned DAG: empty, or with MCP_STUB_PLAN_NODES=n a chain
    over the first n registry services (a response the size of a real plan)."""
    import os
    n = int(os.environ.get("MCP_STUB_PLAN_NODES", "0") or 0)
    if n <= 0:
        return None
    svcs = registry.list_services()[:n]
    nodes = [{"name": s["name"], "endpoint": s["endpoint"],
              "inputs": {"x": svcs[i - 1]["name"] if i else "payload"}}
             for i, s in enumerate(svcs)]
    edges = [{"from": a["name"], "to": b["name"]} for a, b in zip(svcs, svcs[1:])]
    return {"nodes": nodes, "edges": edges}


def replica_config(settings: Settings, registry: BaseRegistry):
    """The replica processes' configuration from the settings."""
    from ..parallel.router import ReplicaConfig
    cfg = ReplicaConfig(model=settings.model, max_batch=settings.max_batch,
                        max_nodes=settings.max_nodes, min_nodes=settings.min_nodes,
                        seed=settings.seed, num_blocks=settings.kv_blocks or None,
                        max_step_tokens=settings.max_step_tokens,
                        temperature=settings.temperature,
                        retrieval_threshold=settings.retrieval_threshold,
                        topk=settings.topk, embed_dim=settings.embed_dim,
                        tp=max(1, int(settings.tp)))
    from ..registry import RedisRegistry
    if isinstance(registry, RedisRegistry):
        cfg.redis_url, cfg.services_prefix = registry.client.url, registry.prefix
    if settings.model == "stub":
        # stub replicas (no engine): MCP_STUB_LATENCY_MS per intent,
        # MCP_STUB_STALL="at_s:stall_s" freezes each replica once
        import os
        stall = os.environ.get("MCP_STUB_STALL", "")
        at, _, dur = stall.partition(":")
        cfg.stub_latency_s = float(os.environ.get("MCP_STUB_LATENCY_MS", "0") or 0) / 1e3
        cfg.stub_stall_at = float(at) if stall else -1.0
        cfg.stub_stall_s = float(dur or 0)
        cfg.stub_plan = _stub_plan(registry, settings)
    return cfg


def build_planner(settings: Settings, registry: BaseRegistry,
                  planner_transport: Optional[httpx.AsyncBaseTransport] = None) -> Planner:
    """The planner backend ``settings`` name: stub, a local engine (one
    process, a TP group, or DP replicas behind a router), or a hosted
    OpenAI-compatible endpoint."""
    if settings.planner_backend == "local":
        if settings.replicas > 1 or settings.router:
            # request-level DP over replicas, each a TP group of
            # settings.tp ranks (MCP_REPLICAS=2 MCP_TP=4: two TP=4 planners);
            # several API workers share the supervisor's replicas instead
            # (serve(): SharedReplicas + SharedRouter)
            from ..parallel.router import ReplicaRouter, group_devices
            cfg = replica_config(settings, registry)
            groups = replica_slice(group_devices(settings.replicas, cfg.tp), settings.replica_slice)
            return ReplicaRouter(groups, settings.model, registry, config=cfg)
        if settings.tp > 1:
            # this process becomes TP rank 0 (driver); ranks 1..tp-1 are
            # spawned worker processes (parallel/tp_serve.py)
            from ..parallel.tp_serve import TPPlanner
            return TPPlanner.launch(settings, registry)
        from ..planner.local import LocalPlanner
        return LocalPlanner.from_settings(settings, registry)
    if settings.planner_backend == "openai":
        from ..planner.remote import RemotePlanner
        return RemotePlanner(registry, settings.openai_base_url, settings.openai_api_key,
                             settings.remote_model, settings.temperature,
                             transport=planner_transport)
    return StubPlanner(registry)


def make_registry_from(settings: Settings) -> BaseRegistry:
    registry = make_registry(settings.redis_url, settings.services_prefix)
    if settings.synthetic_services > 0 and not settings.redis_url:
        from ..registry import synthetic_registry
        registry.register_many(synthetic_registry(settings.synthetic_services, seed=1))
    return registry


def create_app(settings: Optional[Settings] = None, registry: Optional[BaseRegistry] = None,
               planner: Optional[Planner] = None,
               transport: Optional[httpx.AsyncBaseTransport] = None,
               planner_transport: Optional[httpx.AsyncBaseTransport] = None,
               settle_gc: bool = False) -> FastAPI:
    """``settle_gc``: after start-up, move the heap to the permanent GC
    generation (``utils/heap.py``) - for a serving process's entry point only
    (``main``, ``uvicorn ...:app``), never for apps built inside a library or
    a test process, where frozen objects would never be collected."""
    settings = settings or Settings.from_env()
    if registry is None:
        registry = make_registry_from(settings)
    state = {}

    def _make_planner() -> Planner:
        if planner is not None:
            return planner
        return build_planner(settings, registry, planner_transport)

    @contextlib.asynccontextmanager
    async def lifespan(app: FastAPI):
        client = httpx.AsyncClient(transport=transport) if transport is not None else httpx.AsyncClient()
        state["orch"] = Orchestrator(client=client, timeout=settings.exec_timeout,
                                     retries=settings.retries,
                                     concurrent_generations=settings.concurrent_generations,
                                     registry=registry,
                                     use_registry_fallback=settings.use_registry_fallback,
                                     telemetry_to_registry=settings.telemetry_to_registry)
        state["planner"] = _make_planner()
        if settings.plan_cache > 0:
            from ..planner.base import CachedPlanner
            state["planner"] = CachedPlanner(state["planner"], registry, settings.plan_cache)
        if settings.adaptive:        # outside the cache: fresh telemetry applies to cached plans
            from ..planner.audit import AdaptivePlanner
            state["planner"] = AdaptivePlanner(state["planner"], registry,
                                               settings.adaptive_error_rate,
                                               settings.adaptive_min_calls,
                                               settings.adaptive_retries)
        if settle_gc:
            from ..utils.heap import settle
            settle()                       # start-up heap -> permanent GC generation
        try:
            yield
        finally:
            await state["planner"].aclose()
            await client.aclose()

    app = FastAPI(lifespan=lifespan)
    app.state.registry = registry
    app.state.settings = settings
    app.state.components = state

    async def _plan(intent: str) -> dict:
        try:
            return await state["planner"].plan(intent)
        except RuntimeError as e:
            if type(e).__name__ == "EngineStalled":       # hung GPU step: retry elsewhere
                raise HTTPException(status_code=503, detail=str(e))
            raise

    def _explain(graph: dict) -> str:
        from ..planner.audit import explain_plan
        return explain_plan(graph, registry, settings.retries, settings.use_registry_fallback)

    @app.post("/plan", response_model=PlanResponse)
    async def plan_intent(req: PlanRequest):
        graph = await _plan(req.intent)
        if not req.explain:
            # the validated model serialised once, straight into the response:
            # FastAPI's response_model pass would validate and encode it again
            # (~1/4 of the API process's time per plan at thousands of plans/s)
            return Response(plan_response_json(graph), media_type="application/json")
        resp = PlanResponse(graph=graph)                     # a non-object plan -> 500 (T8)
        try:
            text = _explain(resp.graph)
        except Exception as e:     # a plan the orchestrator would reject (T2 / cycle)
            text = f"plan cannot be executed: {type(e).__name__}: {e}"
        return JSONResponse({"graph": resp.graph, "explanation": text})

    @app.post("/explain", response_model=ExplainResponse)
    async def explain_graph(req: ExplainRequest):
        try:
            return ExplainResponse(explanation=_explain(req.graph))
        except Exception as e:
            raise HTTPException(status_code=422, detail=f"{type(e).__name__}: {e}")

    @app.post("/execute", response_model=ExecuteResponse)
    async def run_graph(req: ExecuteRequest):
        return ExecuteResponse(**await state["orch"].execute(req.graph, req.payload))

    @app.post("/plan_and_execute", response_model=ExecuteResponse)
    async def plan_and_run(req: PlanRequest):
        graph = PlanResponse(graph=await _plan(req.intent)).graph
        return ExecuteResponse(**await state["orch"].execute(graph, {}))

    @app.get("/metrics", response_class=PlainTextResponse)
    async def metrics():
        return METRICS.render()

    @app.get("/healthz")
    async def healthz():
        if getattr(state["planner"], "stalled", False):
            raise HTTPException(status_code=503, detail="planner engine stalled")
        return {"ok": True, "services": len(registry.list_services())}

    return app


_APP = None


def __getattr__(name):
    """``uvicorn mcp_amd.api.server:app`` (the reference's
    ``uvicorn control_plane:app``): the app is built from the environment on
    first access, not at import, so importing the module opens no connection
    and loads no model (the reference built its singletons at import, :135-138)."""
    global _APP
    if name == "app":
        if _APP is None:
            _APP = create_app(settle_gc=True)     # a server process's own app
        return _APP
    raise AttributeError(name)


def _reuseport_socket(host: str, port: int):
    import socket
    fam = socket.AF_INET6 if ":" in host else socket.AF_INET
    sock = socket.socket(fam, socket.SOCK_STREAM)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    sock.bind((host, port))
    sock.listen(2048)
    sock.set_inheritable(True)
    return sock


def _api_worker(idx: int, n: int, host: str, port: int, access_log: bool,
                http: str = "fast", shared=None):  # pragma: no cover - process entry
    """One API worker process: builds its planner BEFORE it binds, so the
    kernel never hands a connection to a worker that is still loading; then
    serves on its own SO_REUSEPORT socket.  With the local planner the
    planner is a ``SharedRouter`` over the supervisor's replicas (every
    worker may dispatch to every replica); otherwise each worker builds its
    own (stub / remote backends)."""
    settings = Settings.from_env()
    registry = make_registry_from(settings)
    if shared is not None:
        from ..parallel.router import SharedRouter
        planner = SharedRouter(shared, idx, registry)
    else:
        planner = build_planner(settings, registry)
    app = create_app(settings, registry=registry, planner=planner, settle_gc=True)
    sock = _reuseport_socket(host, port)
    msg = f"mcp api worker {idx}/{n} ready on {host}:{port} ({http})"
    if http == "fast":
        import asyncio
        from .fasthttp import serve_fast
        prof_dir = os.environ.get("MCP_PROFILE_DIR")   # diagnostics: cProfile each API worker
        if prof_dir:
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
            try:
                asyncio.run(serve_fast(app, sock=sock, ready=lambda: print(msg, flush=True)))
            finally:
                prof.disable()
                prof.dump_stats(os.path.join(prof_dir, f"api-worker-{idx}.prof"))
            return
        asyncio.run(serve_fast(app, sock=sock, ready=lambda: print(msg, flush=True)))
        return
    import uvicorn
    server = uvicorn.Server(uvicorn.Config(app, host=host, port=port, access_log=access_log))
    print(msg, flush=True)
    server.run(sockets=[sock])


def check_worker_layout(settings: Settings, workers: int) -> None:
    """Several API workers with the local planner must split the node's
    replicas between them (the router path): without it every worker would
    build its own engine (or TP group) on the same GPU(s), N engines sizing
    their KV pools from the same free HBM.  Raises SystemExit otherwise."""
    if workers <= 1 or settings.planner_backend != "local":
        return
    if not (settings.replicas > 1 or settings.router):
        raise SystemExit(f"--workers {workers} with the local planner needs the replica router "
                         f"(MCP_REPLICAS >= {workers}, or MCP_ROUTER=1 with enough replicas): "
                         "each API worker would otherwise load its own engine on the same GPU")
    if workers > settings.replicas:
        raise SystemExit(f"--workers {workers} > MCP_REPLICAS {settings.replicas}: "
                         "every API worker routes to at least one replica")


def serve(host: str, port: int, workers: int = 1, access_log: bool = True,
          max_restarts: int = 3, http: str = "fast") -> int:  # pragma: no cover - process entry
    """Run the API.  ``http``: "fast" (api/fasthttp.py: own HTTP/1.1 parser,
    /plan answered straight from the planner, everything else through the
    FastAPI app) or "uvicorn" (the reference's server).  ``workers`` > 1: a
    supervisor (which never touches the GPU) spawns that many API worker
    processes on one SO_REUSEPORT port; the kernel spreads connections over
    them, each worker parses HTTP and routes to its own contiguous slice of
    the node's planner replicas (MCP_REPLICAS / MCP_TP), so no single process
    carries every request of the node.  A worker that dies is restarted (its
    replicas with it) up to ``max_restarts`` times."""
    if workers <= 1:
        if http == "fast":
            import asyncio
            from .fasthttp import serve_fast
            asyncio.run(serve_fast(create_app(settle_gc=True), host=host, port=port,
                                   ready=lambda: print(f"mcp api ready on {host}:{port} (fast)",
                                                       flush=True)))
            return 0
        import uvicorn

        class _Server(uvicorn.Server):
            async def startup(self, sockets=None):
                await super().startup(sockets=sockets)
                if self.started:         # the same ready line as the other modes
                    print(f"mcp api ready on {host}:{port} (uvicorn)", flush=True)

        _Server(uvicorn.Config(create_app(settle_gc=True), host=host, port=port,
                               access_log=access_log)).run()
        return 0
    import multiprocessing as mp
    import signal
    import time
    settings = Settings.from_env()
    check_worker_layout(settings, workers)
    ctx = mp.get_context("spawn")
    procs = {}
    restarts = [0] * workers
    shared = None
    if settings.planner_backend == "local":
        # the node's replicas belong to this supervisor (which never touches
        # the GPU itself) and are shared by every worker: request-level
        # least-loaded dispatch whichever worker a connection landed on
        from ..parallel.router import SharedReplicas, ensure_metrics_dir, group_devices
        ensure_metrics_dir()
        registry = make_registry_from(settings)
        cfg = replica_config(settings, registry)
        shared = SharedReplicas(group_devices(settings.replicas, cfg.tp), cfg, registry, workers)
        shared.start()

    def start(i):
        p = ctx.Process(target=_api_worker, args=(i, workers, host, port, access_log, http,
                                                  shared), name=f"mcp-api-{i}")
        p.start()
        procs[i] = p

    stopping = []

    def stop(signum, frame):
        stopping.append(signum)

    signal.signal(signal.SIGTERM, stop)
    signal.signal(signal.SIGINT, stop)
    for i in range(workers):
        start(i)
    rc = 0
    while not stopping:
        time.sleep(0.2)
        for i, p in list(procs.items()):
            if not p.is_alive() and not stopping:
                if restarts[i] >= max_restarts:
                    stopping.append("dead")
                    rc = 1
                    break
                restarts[i] += 1
                if shared is not None:
                    shared.reset_worker(i)
                start(i)
    for p in procs.values():
        if p.is_alive():
            p.terminate()
    for p in procs.values():
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    if shared is not None:
        shared.close()
    return rc


def main():  # pragma: no cover - CLI entry (reference :155-157)
    import argparse
    import os
    ap = argparse.ArgumentParser(description="MI355X MCP control plane")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--workers", type=int, default=int(os.environ.get("MCP_API_WORKERS", "1")),
                    help="API worker processes on one SO_REUSEPORT port (MCP_API_WORKERS)")
    ap.add_argument("--http", choices=["fast", "uvicorn"], default=os.environ.get("MCP_HTTP", "fast"),
                    help="front end: the lean HTTP/1.1 server (api/fasthttp.py) or uvicorn")
    ap.add_argument("--no-access-log", action="store_true",
                    help="skip uvicorn's per-request access log line")
    args = ap.parse_args()
    raise SystemExit(serve(args.host, args.port, args.workers, not args.no_access_log,
                           http=args.http))


if __name__ == "__main__":  # pragma: no cover
    main()
