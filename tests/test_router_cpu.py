"""DP replica router on CPU: least-loaded dispatch over 2 replica processes,
and draining a killed replica."""
import asyncio

import pytest

from mcp_amd.orchestrator import validate_dag
from mcp_amd.parallel.router import ReplicaRouter
from mcp_amd.planner.prompt import synthetic_intent
from mcp_amd.registry import MemoryRegistry, synthetic_registry


@pytest.mark.timeout(600)
def test_router_dispatch_and_failover():
    reg = MemoryRegistry(synthetic_registry(4, seed=11))
    names = [s.name for s in reg.list_services()]
    router = ReplicaRouter(["cpu", "cpu"], "tiny", reg, max_batch=8, max_nodes=3, num_blocks=256,
                           request_timeout=300)

    async def go():
        dags = await asyncio.gather(*[router.plan(synthetic_intent(i)) for i in range(4)])
        for d in dags:
            validate_dag(d, names)
        router.kill_replica(0)
        await asyncio.sleep(0.5)
        more = await asyncio.gather(*[router.plan(synthetic_intent(10 + i)) for i in range(3)])
        for d in more:
            validate_dag(d, names)
        assert router.alive == [False, True]
        await router.aclose()
    asyncio.run(go())
