"""Plan explanations and telemetry-adaptive plans (README.md:43-44,48,50 claims
that control_plane.py never implements; planner/audit.py)."""
import asyncio
import json

import httpx
from fastapi.testclient import TestClient

from mcp_amd.api.server import create_app
from mcp_amd.config import Settings
from mcp_amd.orchestrator import Orchestrator
from mcp_amd.planner.audit import AdaptivePlanner, adapt_plan, explain_plan, fallback_chain
from mcp_amd.planner.base import StubPlanner
from mcp_amd.registry import MemoryRegistry, make_service

GRAPH = {"nodes": [{"name": "d", "endpoint": "http://d/api", "inputs": {"x": "b", "y": "c"}},
                   {"name": "c", "endpoint": "http://c/api", "inputs": {"x": "a"}},
                   {"name": "b", "endpoint": "http://b/api", "inputs": {"x": "a"}, "retries": 2},
                   {"name": "a", "endpoint": "http://a/api", "inputs": {"u": "user_id"}}],
         "edges": [{"from": "a", "to": "b", "fallback": "http://b-fb/api"},
                   {"from": "a", "to": "c"}, {"from": "b", "to": "d"}, {"from": "c", "to": "d"}]}


def registry():
    recs = [make_service(n, {"x": "string"}, {"y": "string"}, cost=0.01) for n in "abcd"]
    for r in recs:
        r["fallback"] = f"http://{r['name']}-reg-fb/api"
    return MemoryRegistry(recs)


def test_explanation_follows_execution_order_and_fallbacks():
    reg = registry()
    text = explain_plan(GRAPH, reg)
    order = [text.index(f"{n}. {s} ->") for n, s in zip(range(1, 5), "abcd")]
    assert order == sorted(order)                       # T3 generational order a, b, c, d
    assert "Stage 2 (independent steps" in text
    assert "payload field 'user_id'" in text
    assert "the full response of step 'b'" in text
    assert "2 retries, then fallbacks in order: http://b-fb/api" in text
    assert "no fallback, the whole request aborts with HTTP 502" in text   # a, c, d
    assert "Estimated cost: 0.04 (4 of 4" in text
    # the registry fallback only counts when the orchestrator would use it
    assert fallback_chain(GRAPH, "c", reg, use_registry_fallback=True) == ["http://c-reg-fb/api"]
    assert explain_plan(GRAPH, reg) == text             # deterministic


def test_explanation_includes_telemetry():
    reg = registry()
    for ok in (True, True, False, True):
        reg.record_call("a", 0.010, ok)
    assert "telemetry: 4 call(s), error rate 25.0%, mean latency 10.0 ms" in explain_plan(GRAPH, reg)


def test_adapt_plan_hardens_failing_services_only():
    reg = registry()
    for _ in range(6):
        reg.record_call("c", 0.01, False)
    reg.record_call("b", 0.01, False)                   # too few calls to judge
    for _ in range(10):
        reg.record_call("d", 0.01, True)
    out = adapt_plan(GRAPH, reg, error_rate=0.2, min_calls=5, retries=1)
    nodes = {n["name"]: n for n in out["nodes"]}
    assert nodes["c"]["retries"] == 1 and nodes["c"]["fallbacks"] == ["http://c-reg-fb/api"]
    assert "error rate 100.0% over 6 calls" in nodes["c"]["adapted"]
    for n in "abd":
        assert "adapted" not in nodes[n]
    assert GRAPH["nodes"][1] == {"name": "c", "endpoint": "http://c/api", "inputs": {"x": "a"}}
    assert [n["name"] for n in out["nodes"]] == [n["name"] for n in GRAPH["nodes"]]


def test_adapted_plan_recovers_through_registry_fallback():
    """A service with a bad record gets its registry fallback added; the
    orchestrator then completes the plan instead of returning 502."""
    reg = registry()
    for _ in range(5):
        reg.record_call("c", 0.01, False)

    def h(request):
        if request.url.host == "c":
            return httpx.Response(503)
        return httpx.Response(200, json={"svc": request.url.host})

    async def run(graph):
        orch = Orchestrator(client=httpx.AsyncClient(transport=httpx.MockTransport(h)))
        try:
            return await orch.execute(graph, {"user_id": 1})
        finally:
            await orch.client.aclose()

    plain = {"nodes": [{"name": "c", "endpoint": "http://c/api", "inputs": {}}], "edges": []}
    try:
        asyncio.run(run(plain))
        raise AssertionError("expected 502")
    except Exception as e:
        assert getattr(e, "status_code", None) == 502
    out = asyncio.run(run(adapt_plan(plain, reg)))
    assert out["results"]["c"] == {"svc": "c-reg-fb"}
    assert "503" in out["errors"]["c"]


def test_api_explain_and_adaptive():
    reg = registry()
    for _ in range(5):
        reg.record_call("a", 0.01, False)

    def h(request):
        return httpx.Response(200, json={"svc": request.url.host})

    app = create_app(Settings(adaptive=True), registry=reg, planner=StubPlanner(reg, canned=GRAPH),
                     transport=httpx.MockTransport(h))
    with TestClient(app, raise_server_exceptions=False) as c:
        r = c.post("/plan", json={"intent": "x"})
        assert r.status_code == 200 and set(r.json()) == {"graph"}      # wire parity by default
        a = {n["name"]: n for n in r.json()["graph"]["nodes"]}["a"]
        assert a["fallbacks"] == ["http://a-reg-fb/api"] and a["retries"] == 1
        r = c.post("/plan", json={"intent": "x", "explain": True})
        assert set(r.json()) == {"graph", "explanation"}
        assert "fallbacks in order: http://a-reg-fb/api" in r.json()["explanation"]
        r = c.post("/explain", json={"graph": GRAPH})
        assert r.status_code == 200 and r.json()["explanation"].startswith("Plan with 4 step(s)")
        cyc = {"nodes": [{"name": "p", "endpoint": "e", "inputs": {}},
                         {"name": "q", "endpoint": "e", "inputs": {}}],
               "edges": [{"from": "p", "to": "q"}, {"from": "q", "to": "p"}]}
        assert c.post("/explain", json={"graph": cyc}).status_code == 422
        assert c.post("/explain", json={"graph": {"nodes": []}}).status_code == 422


def test_adaptive_planner_passes_malformed_output_through():
    reg = registry()
    p = AdaptivePlanner(StubPlanner(reg, canned="[1, 2]"), reg)
    assert asyncio.run(p.plan("x")) == [1, 2]
    assert json.dumps(asyncio.run(AdaptivePlanner(StubPlanner(reg, canned=GRAPH), reg).plan("x"))) \
        == json.dumps(GRAPH)
