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
        registry = make_registry(settings.redis_url, settings.services_prefix)
        if settings.synthetic_services > 0 and not settings.redis_url:
            from ..registry import synthetic_registry
            registry.register_many(synthetic_registry(settings.synthetic_services, seed=1))
    state = {}

    def _make_planner() -> Planner:
        if planner is not None:
            return planner
        if settings.planner_backend == "local":
            if settings.replicas > 1 or settings.router:
                # request-level DP over replicas, each a TP group of
                # settings.tp ranks (MCP_REPLICAS=2 MCP_TP=4: two TP=4 planners)
                from ..parallel.router import ReplicaConfig, ReplicaRouter, group_devices
                cfg = ReplicaConfig(model=settings.model, max_batch=settings.max_batch,
                                    max_nodes=settings.max_nodes, min_nodes=settings.min_nodes,
                                    seed=settings.seed,
                                    num_blocks=settings.kv_blocks or None,
                                    max_step_tokens=settings.max_step_tokens,
                                    temperature=settings.temperature,
                                    retrieval_threshold=settings.retrieval_threshold,
                                    topk=settings.topk, embed_dim=settings.embed_dim,
                                    tp=max(1, int(settings.tp)))
                return ReplicaRouter(group_devices(settings.replicas, cfg.tp), settings.model,
                                     registry, config=cfg)
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
        resp = PlanResponse(graph=await _plan(req.intent))   # a non-object plan -> 500 (T8)
        if not req.explain:
            # the validated model serialised once, straight into the response:
            # FastAPI's response_model pass would validate and encode it again
            # (~1/4 of the API process's time per plan at thousands of plans/s)
            return Response(resp.__pydantic_serializer__.to_json(resp), media_type="application/json")
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


def main():  # pragma: no cover - CLI entry (reference :155-157)
    import argparse

    import uvicorn
    ap = argparse.ArgumentParser(description="MI355X MCP control plane")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--no-access-log", action="store_true",
                    help="skip uvicorn's per-request access log line")
    args = ap.parse_args()
    uvicorn.run(create_app(settle_gc=True), host=args.host, port=args.port, access_log=not args.no_access_log)


if __name__ == "__main__":  # pragma: no cover
    main()
