"""``MCP_TP=2`` behind the API on CPU (gloo): the API process is TP rank 0
(driver: scheduler, grammar, sampling), one spawned worker process mirrors
the sharded forward; /plan returns valid T2 DAGs and shutdown releases the
worker (SURVEY §2.3 TP; the reference's /plan, control_plane.py:140-142)."""
import httpx
import pytest
from fastapi.testclient import TestClient

from mcp_amd.api.server import create_app
from mcp_amd.config import Settings
from mcp_amd.orchestrator import validate_dag
from mcp_amd.registry import MemoryRegistry, synthetic_registry


@pytest.mark.timeout(600)
def test_plan_with_tp2_on_gloo(monkeypatch):
    monkeypatch.setenv("MCP_TP_DEVICES", "cpu,cpu")
    reg = MemoryRegistry(synthetic_registry(6, seed=2))
    names = [s.name for s in reg.list_services()]
    st = Settings(planner_backend="local", model="tiny-tp", tp=2, max_batch=8,
                  max_step_tokens=2048, max_nodes=3, kv_blocks=256)

    def h(request):
        return httpx.Response(200, json={"ok": True})
    app = create_app(st, registry=reg, transport=httpx.MockTransport(h))
    with TestClient(app) as c:
        planner = app.state.components["planner"]
        assert type(planner).__name__ == "TPPlanner" and planner.engine.model.tp == 2
        for i in range(3):
            r = c.post("/plan", json={"intent": f"look up user {i} and charge the order"})
            assert r.status_code == 200, r.text
            validate_dag(r.json()["graph"], names)
        r = c.post("/plan_and_execute", json={"intent": "refund the order"})
        assert r.status_code in (200, 502), r.text
        workers = list(planner._workers)
    for p in workers:                       # lifespan exit stopped the worker rank
        assert not p.is_alive() and p.exitcode == 0
