"""Engine routing of long-context, low-batch decode steps to split-KV
attention (K6): a ~6k-token prompt (90-service registry, no retrieval
pruning) planned greedily with split-KV on and off gives the same DAG, and
the split path actually ran."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(300)
def test_long_context_decode_uses_split_kv(monkeypatch):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from mcp_amd.engine.engine import LLMEngine
    from mcp_amd.models.llama import LlamaModel
    from mcp_amd.orchestrator import validate_dag
    from mcp_amd.planner.local import LocalPlanner
    from mcp_amd.planner.prompt import synthetic_intent
    from mcp_amd.registry import MemoryRegistry, synthetic_registry

    reg = MemoryRegistry(synthetic_registry(90, seed=4))
    names = [s.name for s in reg.list_services()]
    model = LlamaModel.random("llama3-1b-ish", "cuda:0", seed=3)
    out = {}
    for mode in ("0", "-1"):
        monkeypatch.setenv("MCP_KV_SPLIT", mode)
        eng = LLMEngine(model, num_blocks=1024, max_batch=4, max_step_tokens=8192,
                        temperature=0.0)
        pl = LocalPlanner(eng, reg, max_nodes=4, retrieval_threshold=10 ** 6)
        dec, ptoks, stoks = pl.prepare(synthetic_intent(3))
        assert len(ptoks) + len(stoks) > 4096
        dags = pl.plan_many([synthetic_intent(3)])
        validate_dag(dags[0], names)
        out[mode] = (dags[0], eng.stats["kv_split_steps"])
        torch.cuda.synchronize()
    assert out["0"][1] == 0 and out["-1"][1] > 0
    assert out["0"][0] == out["-1"][0]
