"""API (T8, 422/500/502) and registry (T1, RESP backend) contract tests."""
import asyncio
import json

import httpx
import pytest
from fastapi.testclient import TestClient

from mcp_amd.api.server import create_app
from mcp_amd.config import Settings
from mcp_amd.planner.base import StubPlanner
from mcp_amd.planner.prompt import build_prompt, build_prompt_parts
from mcp_amd.registry import (MemoryRegistry, RedisRegistry, RespClient, RespServer,
                              make_service, synthetic_registry)


def services3():
    return [make_service("user-profile", {"user_id": "string"}, {"profile": "object"}),
            make_service("order-quote", {"profile": "object"}, {"quote": "number"}),
            make_service("email-notify", {"quote": "number"}, {"status": "string"})]


def mock_transport():
    def h(request):
        return httpx.Response(200, json={"svc": request.url.host, "in": json.loads(request.content)})
    return httpx.MockTransport(h)


def client_for(planner=None, registry=None):
    reg = registry or MemoryRegistry(services3())
    app = create_app(Settings(), registry=reg, planner=planner or StubPlanner(reg),
                     transport=mock_transport())
    return TestClient(app, raise_server_exceptions=False)


def test_plan_execute_roundtrip():
    with client_for() as c:
        r = c.post("/plan", json={"intent": "look up the user profile and quote the order"})
        assert r.status_code == 200
        g = r.json()["graph"]
        assert {n["name"] for n in g["nodes"]} <= {"user-profile", "order-quote", "email-notify"}
        r2 = c.post("/execute", json={"graph": g, "payload": {"user_id": "u1"}})
        assert r2.status_code == 200 and set(r2.json()) == {"results", "errors"}
        r3 = c.post("/plan_and_execute", json={"intent": "email the user"})
        assert r3.status_code == 200
        assert c.get("/metrics").text.count("mcp_") > 0


def test_missing_intent_422_and_bad_plans_500():
    with client_for() as c:
        assert c.post("/plan", json={}).status_code == 422
    with client_for(planner=StubPlanner(canned="```json\n{}\n```")) as c:
        assert c.post("/plan", json={"intent": "x"}).status_code == 500
    with client_for(planner=StubPlanner(canned="[1, 2]")) as c:
        assert c.post("/plan", json={"intent": "x"}).status_code == 500
    with client_for(planner=StubPlanner(canned={})) as c:        # {} plan -> KeyError('nodes')
        assert c.post("/plan_and_execute", json={"intent": "x"}).status_code == 500


def test_plan_and_execute_uses_empty_payload():
    canned = {"nodes": [{"name": "a", "endpoint": "http://a/api", "inputs": {"k": "uid"}}], "edges": []}
    with client_for(planner=StubPlanner(canned=canned)) as c:
        r = c.post("/plan_and_execute", json={"intent": "x"})
        assert r.json()["results"]["a"]["in"] == {"k": None}


def test_502_detail():
    def h(request):
        return httpx.Response(500)
    reg = MemoryRegistry(services3())
    app = create_app(Settings(), registry=reg, planner=StubPlanner(reg), transport=httpx.MockTransport(h))
    with TestClient(app, raise_server_exceptions=False) as c:
        g = {"nodes": [{"name": "a", "endpoint": "http://a/api", "inputs": {}}], "edges": []}
        r = c.post("/execute", json={"graph": g, "payload": {}})
        assert r.status_code == 502
        assert r.json() == {"detail": "a failed and no fallback available"}


def test_memory_registry_sorted_and_versioned():
    reg = MemoryRegistry()
    v0 = reg.version
    for s in reversed(services3()):
        reg.register(s)
    assert [s.name for s in reg.list_services()] == sorted(s["name"] for s in services3())
    assert reg.version == v0 + 3
    assert reg.unregister("order-quote") and reg.version == v0 + 4


def test_resp_registry_roundtrip():
    with RespServer() as url:
        reg = RedisRegistry(url)
        recs = synthetic_registry(40)
        reg.register_many(recs)
        got = reg.list_services()
        assert [r.name for r in got] == sorted(r["name"] for r in recs)
        assert got[0] == sorted(recs, key=lambda r: r["name"])[0]          # T1 byte-exact fields
        # raw record layout under the reference key prefix
        cl = RespClient(url)
        raw = cl.get("mcp:service:" + recs[0]["name"])
        assert json.loads(raw) == recs[0]
        cl.delete("mcp:service:" + recs[1]["name"])
        assert len(reg.list_services()) == 39
        reg.record_call("x", 0.25, False)
        reg.record_call("x", 0.75, True)
        t = reg.telemetry("x")
        assert t["calls"] == 2 and t["errors"] == 1 and abs(t["latency_sum"] - 1.0) < 1e-6
        assert reg.version >= 1


def test_prompt_parts_share_prefix():
    svcs = services3()
    p1, s1 = build_prompt_parts(svcs, "a")
    p2, s2 = build_prompt_parts(svcs, "b")
    assert p1 == p2 and s1 != s2
    full = build_prompt(svcs, "a")
    assert full == p1 + s1
    assert "\\n" not in full and "“a”" in full and full.endswith("JSON DAG:")


def test_openai_compatible_remote_planner():
    """MCP_PLANNER_BACKEND=openai: the reference's request shape (one system
    message, temperature 0.2, model gpt-4o-mini, bearer key) against a mocked
    /chat/completions; a non-object reply is the reference's HTTP 500."""
    seen = []
    replies = [json.dumps({"nodes": [{"name": "user-profile", "endpoint": "http://user-profile/api",
                                      "inputs": {"user_id": "user_id"}}], "edges": []}),
               "[1, 2]"]

    def llm(request):
        seen.append((str(request.url), request.headers.get("authorization"), json.loads(request.content)))
        return httpx.Response(200, json={"choices": [{"message": {"content": replies[len(seen) - 1]}}]})

    reg = MemoryRegistry(services3())
    st = Settings(planner_backend="openai", openai_base_url="http://llm.test/v1", openai_api_key="k1")
    app = create_app(st, registry=reg, transport=mock_transport(),
                     planner_transport=httpx.MockTransport(llm))
    with TestClient(app, raise_server_exceptions=False) as c:
        r = c.post("/plan", json={"intent": "look up the user"})
        assert r.status_code == 200 and r.json()["graph"]["nodes"][0]["name"] == "user-profile"
        url, auth, body = seen[0]
        assert url == "http://llm.test/v1/chat/completions" and auth == "Bearer k1"
        assert body["model"] == "gpt-4o-mini" and body["temperature"] == 0.2
        assert [m["role"] for m in body["messages"]] == ["system"]
        assert "look up the user" in body["messages"][0]["content"]
        assert c.post("/plan", json={"intent": "x"}).status_code == 500


def test_plan_cache_keyed_by_registry_version():
    """MCP_PLAN_CACHE: repeated intents hit the LRU; a registry change misses."""
    from mcp_amd.planner.base import CachedPlanner
    reg = MemoryRegistry(services3())
    inner = StubPlanner(reg)
    calls = []
    orig = inner.plan

    async def counting(intent):
        calls.append(intent)
        return await orig(intent)
    inner.plan = counting
    cp = CachedPlanner(inner, reg, size=2)
    a = asyncio.run(cp.plan("quote the order"))
    b = asyncio.run(cp.plan("quote the order"))
    assert a == b and len(calls) == 1 and cp.hits == 1
    b["nodes"].clear()                                   # copies: the cache is not mutated
    assert asyncio.run(cp.plan("quote the order")) == a
    reg.register(make_service("new-svc", {"x": "string"}, {"y": "string"}))
    asyncio.run(cp.plan("quote the order"))
    assert len(calls) == 2                               # new registry version: miss
    st = Settings(plan_cache=8)
    app = create_app(st, registry=reg, planner=StubPlanner(reg), transport=mock_transport())
    with TestClient(app) as c:
        r1 = c.post("/plan", json={"intent": "email the user"}).json()
        r2 = c.post("/plan", json={"intent": "email the user"}).json()
        assert r1 == r2 and isinstance(app.state.components["planner"], CachedPlanner)


def test_module_level_app_for_uvicorn(monkeypatch):
    """``uvicorn mcp_amd.api.server:app`` works like the reference's
    ``uvicorn control_plane:app``: a lazily built app from the environment."""
    import importlib

    from fastapi import FastAPI
    monkeypatch.setenv("MCP_PLANNER_BACKEND", "stub")
    monkeypatch.delenv("REDIS_URL", raising=False)
    mod = importlib.import_module("mcp_amd.api.server")
    monkeypatch.setattr(mod, "_APP", None)
    from uvicorn.importer import import_from_string
    app = import_from_string("mcp_amd.api.server:app")
    assert isinstance(app, FastAPI) and app is mod.app
    with TestClient(app) as c:
        assert c.get("/healthz").status_code == 200
        assert c.post("/plan", json={}).status_code == 422
