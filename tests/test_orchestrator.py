"""Contract / parity tests for the DAG executor (§4.3.1).

Downstream services are faked with ``httpx.MockTransport`` (the Probe P1/P6
pattern of SURVEY Appendix A).
"""
import asyncio
import json
import logging

import httpx
import networkx as nx
import pytest
from fastapi import HTTPException

from mcp_amd.orchestrator import Orchestrator, normalize_dag, validate_dag, DagValidationError


def run(coro):
    return asyncio.run(coro)


def make_orch(handler, **kw):
    client = httpx.AsyncClient(transport=httpx.MockTransport(handler))
    return Orchestrator(client=client, **kw)


def echo_handler(calls=None):
    def h(request: httpx.Request):
        body = json.loads(request.content or b"{}")
        if calls is not None:
            calls.append((str(request.url), body))
        return httpx.Response(200, json={"from": request.url.host, "got": body})
    return h


def node(name, inputs=None, **extra):
    d = {"name": name, "endpoint": f"http://{name}/api", "inputs": inputs or {}}
    d.update(extra)
    return d


@pytest.mark.parametrize("nodes,edges,order", [
    (["d", "c", "b", "a"], [("a", "b"), ("a", "c"), ("b", "d"), ("c", "d")], ["a", "b", "c", "d"]),
    (["a", "b", "c", "z"], [("a", "b"), ("b", "c")], ["a", "z", "b", "c"]),
    (["x1", "y1", "x2", "y2"], [("x1", "x2"), ("y1", "y2")], ["x1", "y1", "x2", "y2"]),
])
@pytest.mark.parametrize("concurrent", [False, True])
def test_generational_topo_order(nodes, edges, order, concurrent):
    calls = []
    orch = make_orch(echo_handler(calls), concurrent_generations=concurrent)
    g = {"nodes": [node(n) for n in nodes], "edges": [{"from": a, "to": b} for a, b in edges]}
    out = run(orch.execute(g, {}))
    assert list(out["results"].keys()) == order
    assert out["errors"] == {}
    if not concurrent:
        assert [u.split("/")[2] for u, _ in calls] == order
    # NetworkX itself agrees (T3 is NetworkX's generational Kahn order)
    assert list(nx.topological_sort(Orchestrator.build_graph(g))) == order


def test_input_resolution_whole_body_and_payload():
    orch = make_orch(echo_handler())
    g = {"nodes": [node("a", {"x": "uid"}), node("b", {"y": "a", "q": "missing"})],
         "edges": [{"from": "a", "to": "b"}]}
    out = run(orch.execute(g, {"uid": 7}))
    assert out["results"]["a"] == {"from": "a", "got": {"x": 7}}
    assert out["results"]["b"] == {"from": "b", "got": {"y": {"from": "a", "got": {"x": 7}}, "q": None}}


def failing(status=None, exc=None, nonjson=False, only=None):
    def h(request):
        host = request.url.host
        if only is None or host in only:
            if exc is not None:
                raise exc
            if nonjson:
                return httpx.Response(200, text="not json")
            if status is not None:
                return httpx.Response(status)
        return httpx.Response(200, json={"ok": host})
    return h


def test_http_500_error_string_and_fallback_success(caplog):
    orch = make_orch(failing(status=500, only={"b"}))
    g = {"nodes": [node("a"), node("b")],
         "edges": [{"from": "a", "to": "b", "fallback": "http://b-fallback/api"}]}
    with caplog.at_level(logging.INFO, logger="orchestrator"):
        out = run(orch.execute(g, {}))
    assert out["results"]["b"] == {"ok": "b-fallback"}
    assert out["errors"]["b"] == (
        "Server error '500 Internal Server Error' for url 'http://b/api'\n"
        "For more information check: https://developer.mozilla.org/en-US/docs/Web/HTTP/Status/500")
    msgs = [r.getMessage() for r in caplog.records if r.name == "orchestrator"]
    assert msgs[0].startswith("Service b failed: Server error '500")
    assert msgs[1] == "Attempting fallback http://b-fallback/api for b"


def test_fallback_also_fails_appends():
    def h(request):
        if request.url.host == "b":
            raise httpx.ConnectError("All connection attempts failed")
        if request.url.host == "bf":
            raise httpx.ReadTimeout("timed out")
        return httpx.Response(200, json={})
    orch = make_orch(h)
    g = {"nodes": [node("a"), node("b")], "edges": [{"from": "a", "to": "b", "fallback": "http://bf/api"}]}
    out = run(orch.execute(g, {}))
    assert "b" not in out["results"]
    assert out["errors"]["b"] == "All connection attempts failed; fallback failed: timed out"


def test_non_json_body_is_failure():
    orch = make_orch(failing(nonjson=True, only={"b"}))
    g = {"nodes": [node("a"), node("b")], "edges": [{"from": "a", "to": "b", "fallback": "http://c/api"}]}
    out = run(orch.execute(g, {}))
    assert out["errors"]["b"] == "Expecting value: line 1 column 1 (char 0)"
    assert out["results"]["b"] == {"ok": "c"}


def test_source_node_failure_aborts_502():
    orch = make_orch(failing(status=503, only={"a"}))
    g = {"nodes": [node("a"), node("b")], "edges": [{"from": "a", "to": "b"}]}
    with pytest.raises(HTTPException) as ei:
        run(orch.execute(g, {}))
    assert ei.value.status_code == 502
    assert ei.value.detail == "a failed and no fallback available"


def test_only_first_in_edge_fallback_considered():
    orch = make_orch(failing(status=500, only={"c"}))
    g = {"nodes": [node("a"), node("b"), node("c")],
         "edges": [{"from": "a", "to": "c"}, {"from": "b", "to": "c", "fallback": "http://cf/api"}]}
    with pytest.raises(HTTPException):
        run(orch.execute(g, {}))


@pytest.mark.parametrize("graph,exc", [
    ({"nodes": [node("a")]}, KeyError),                                        # missing edges
    ({"nodes": [node("a")], "edges": [{"from": "a", "to": "ghost"}]}, KeyError),   # unknown node
    ({"nodes": [node("a"), node("b")],
      "edges": [{"from": "a", "to": "b"}, {"from": "b", "to": "a"}]}, nx.NetworkXUnfeasible),
])
def test_malformed_graphs_raise_like_reference(graph, exc):
    orch = make_orch(echo_handler())
    with pytest.raises(exc):
        run(orch.execute(graph, {}))


def test_retries_then_success():
    state = {"n": 0}

    def h(request):
        state["n"] += 1
        if state["n"] < 3:
            return httpx.Response(500)
        return httpx.Response(200, json={"try": state["n"]})
    orch = make_orch(h)
    g = {"nodes": [node("a", retries=2)], "edges": []}
    out = run(orch.execute(g, {}))
    assert out["results"]["a"] == {"try": 3}
    assert "a" in out["errors"]          # the failed attempts are still traced


def test_ordered_node_fallbacks():
    tried = []

    def h(request):
        tried.append(request.url.host)
        if request.url.host in ("a", "f1"):
            return httpx.Response(500)
        return httpx.Response(200, json={"by": request.url.host})
    orch = make_orch(h)
    g = {"nodes": [node("a", fallbacks=["http://f1/api", "http://f2/api"])], "edges": []}
    out = run(orch.execute(g, {}))
    assert tried == ["a", "f1", "f2"]
    assert out["results"]["a"] == {"by": "f2"}
    assert out["errors"]["a"].count("; fallback failed: ") == 1


def test_concurrent_generations_overlap():
    async def slow(request):
        await asyncio.sleep(0.05)
        return httpx.Response(200, json={})
    g = {"nodes": [node(f"n{i}") for i in range(5)], "edges": []}
    import time
    orch = Orchestrator(client=httpx.AsyncClient(transport=httpx.MockTransport(slow)),
                        concurrent_generations=True)
    t0 = time.perf_counter()
    out = run(orch.execute(g, {}))
    t_conc = time.perf_counter() - t0
    assert list(out["results"]) == [f"n{i}" for i in range(5)]
    # relative to the serial executor on the same machine (robust to a loaded CPU):
    # 5 independent 50 ms calls overlap instead of adding up
    serial = Orchestrator(client=httpx.AsyncClient(transport=httpx.MockTransport(slow)))
    t0 = time.perf_counter()
    run(serial.execute(g, {}))
    t_ser = time.perf_counter() - t0
    assert t_ser >= 0.25 and t_conc < 0.6 * t_ser, (t_conc, t_ser)


def test_validate_and_normalize():
    g = {"nodes": [node("a"), node("b")], "edges": [{"from": "a", "to": "b"}]}
    validate_dag(g, ["a", "b"])
    with pytest.raises(DagValidationError):
        validate_dag({"nodes": [node("a")], "edges": [{"from": "a", "to": "a"}]})
    with pytest.raises(DagValidationError):
        validate_dag(g, ["a"])
    t2 = normalize_dag([{"service_name": "a", "endpoint": "http://a/api", "input_keys": ["x"],
                         "next_steps": ["b"], "fallback": "http://fb"},
                        {"service_name": "b", "endpoint": "http://b/api", "input_keys": []}])
    validate_dag(t2)
    assert t2["edges"] == [{"from": "a", "to": "b", "fallback": "http://fb"}]


def test_fast_post_path_matches_client_post(caplog):
    """The orchestrator's fast POST path (client transport, no auth/redirect
    plumbing) gives the same request bytes and headers, the same results,
    the same error strings (HTTP status, redirect, non-JSON body, connection
    error, timeout) and the same httpx INFO line as ``client.post``."""
    seen = {}

    def handler(request: httpx.Request):
        key = request.url.host
        seen.setdefault(key, []).append((request.method, str(request.url),
                                         sorted(request.headers.multi_items()), request.content))
        if key == "err":
            return httpx.Response(500, text="boom")
        if key == "moved":
            return httpx.Response(301, headers={"Location": "http://elsewhere/"})
        if key == "text":
            return httpx.Response(200, text="not json")
        if key == "down":
            raise httpx.ConnectError("All connection attempts failed")
        if key == "slow":
            raise httpx.ReadTimeout("timed out")
        return httpx.Response(200, json={"got": json.loads(request.content), "uni": "é"})

    def outcome(fast):
        o = make_orch(handler)
        if not fast:
            o._fast_ok = lambda: False
        out = []
        for host in ("ok", "err", "moved", "text", "down", "slow"):
            try:
                out.append(("ok", run(o._post(f"http://{host}/api", {"x": 1, "s": "ünï", "n": None}))))
            except Exception as e:  # noqa: BLE001 - compared as text
                out.append((type(e).__name__, str(e)))
        return out

    with caplog.at_level(logging.INFO, logger="httpx"):
        slow = outcome(False)
        n = len(caplog.records)
        fast = outcome(True)
    assert fast == slow
    logs = [r.getMessage() for r in caplog.records if r.name == "httpx"]
    assert logs[:n] == logs[n:] and any('"HTTP/1.1 500 Internal Server Error"' in m for m in logs)
    for host, reqs in seen.items():
        assert reqs[0] == reqs[1], host
    o = make_orch(handler)
    assert o._fast_ok()
    o.client.cookies.set("sid", "1")                 # cookie jars take client.post
    assert not o._fast_ok()


def test_fast_post_path_follows_client_header_changes_and_close():
    """headers set on the client after the first call are
    sent by the fast path (as client.post sends them), and a closed client
    raises client.post's own error."""
    seen = []

    def handler(request: httpx.Request):
        seen.append(dict(request.headers))
        return httpx.Response(200, json={"ok": True})

    o = make_orch(handler)
    assert run(o._post("http://a/api", {"x": 1})) == {"ok": True}
    o.client.headers["X-Trace"] = "t-1"
    run(o._post("http://a/api", {"x": 1}))
    o.client.headers["X-Trace"] = "t-2"
    run(o._post("http://a/api", {"x": 1}))
    assert "x-trace" not in seen[0] and seen[1]["x-trace"] == "t-1" and seen[2]["x-trace"] == "t-2"
    assert o._fast_ok()
    run(o.client.aclose())
    with pytest.raises(RuntimeError, match="client has been closed"):
        run(o._post("http://a/api", {"x": 1}))
