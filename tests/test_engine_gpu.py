"""Engine paths on the GPU: captured hipGraph steps vs eager launches, the
pipelined engine vs the synchronous one, and cascade vs plain attention (all
greedy, so the plans must agree exactly or the DAGs must at least validate)."""
import pytest
import torch

from mcp_amd.engine.engine import LLMEngine
from mcp_amd.models.llama import LlamaModel
from mcp_amd.orchestrator import validate_dag
from mcp_amd.planner.local import LocalPlanner
from mcp_amd.planner.prompt import synthetic_intent
from mcp_amd.registry import MemoryRegistry, synthetic_registry

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _graph_every_bucket(monkeypatch):
    """These tests check the graph machinery on every bucket (copy-on-write,
    cascade and split-KV keys included): lift the serving default that runs
    steps above 128 tokens eagerly (engine._GRAPH_MAX_T); spawned ranks read
    the environment."""
    import mcp_amd.engine.engine as eng_mod
    monkeypatch.setenv("MCP_GRAPH_MAX_TOKENS", "1000000")
    monkeypatch.setattr(eng_mod, "_GRAPH_MAX_T", 1000000)


def _plans(model, reg, intents, **kw):
    eng = LLMEngine(model, num_blocks=512, max_batch=32, temperature=0.0, **kw)
    planner = LocalPlanner(eng, reg, max_nodes=4, min_nodes=2)
    out = planner.plan_many(intents)
    assert eng.alloc.num_free == eng.kv.num_blocks
    return out, eng


@pytest.mark.parametrize("cascade", [False, True])
def test_graph_replay_matches_eager(cascade):
    model = LlamaModel.random("tiny", "cuda", seed=3)
    reg = MemoryRegistry(synthetic_registry(8, seed=2))
    intents = [synthetic_intent(i) for i in range(6)]
    eager, e1 = _plans(model, reg, intents, graphs=False, cascade=cascade, pipeline=False)
    graph, e2 = _plans(model, reg, intents, graphs=True, cascade=cascade, pipeline=False)
    assert e2.stats["graph_steps"] > 0 and e1.stats["graph_steps"] == 0
    # prefix copy-on-write steps (requests attaching to the shared registry
    # prefix) replay too, and nearly every step is graphed
    assert e2.stats["graph_cow_steps"] > 0
    assert e2.stats["graph_steps"] >= 0.8 * e2.stats["steps"], e2.stats
    assert graph == eager
    names = [s.name for s in reg.list_services()]
    for d in graph:
        validate_dag(d, names)


def test_pipelined_and_cascade_paths_valid():
    model = LlamaModel.random("llama3-1b-ish", "cuda", seed=4)
    reg = MemoryRegistry(synthetic_registry(10, seed=1))
    intents = [synthetic_intent(i) for i in range(40)]
    names = [s.name for s in reg.list_services()]
    a, _ = _plans(model, reg, intents, graphs=False, cascade=False, pipeline=False)
    b, eb = _plans(model, reg, intents, graphs=True, cascade=True, pipeline=True)
    for d in a + b:
        validate_dag(d, names)
    # greedy decoding: identical choices unless bf16 rounding differs between
    # the cascade (LSE-merged) and plain attention paths; require broad agreement
    same = sum(x == y for x, y in zip(a, b))
    assert same >= len(a) * 0.8, same


def test_api_local_planner_end_to_end():
    """FastAPI app with the on-GPU planner (tiny Llama shapes, same kernels):
    concurrent /plan requests through the async engine thread, /plan_and_execute
    against mocked services, /healthz and /metrics."""
    import asyncio
    import json

    import httpx
    from fastapi.testclient import TestClient

    from mcp_amd.api.server import create_app
    from mcp_amd.config import Settings

    reg = MemoryRegistry(synthetic_registry(6, seed=5))
    names = [s.name for s in reg.list_services()]

    def h(request):
        return httpx.Response(200, json={"svc": request.url.host, "in": json.loads(request.content)})

    st = Settings(planner_backend="local", model="tiny", max_batch=16, max_step_tokens=2048,
                  kv_blocks=256, max_nodes=4, embed_dim=256)
    app = create_app(st, registry=reg, transport=httpx.MockTransport(h))
    with TestClient(app, raise_server_exceptions=False) as c:
        assert c.get("/healthz").json()["ok"]

        async def many():
            transport = httpx.ASGITransport(app=app)
            async with httpx.AsyncClient(transport=transport, base_url="http://t") as ac:
                rs = await asyncio.gather(*[ac.post("/plan", json={"intent": synthetic_intent(i)})
                                            for i in range(8)])
            return rs

        for r in asyncio.run(many()):
            assert r.status_code == 200
            validate_dag(r.json()["graph"], names)
        r = c.post("/plan_and_execute", json={"intent": synthetic_intent(99)})
        assert r.status_code == 200 and set(r.json()) == {"results", "errors"}
        m = c.get("/metrics")
        assert m.status_code == 200 and "mcp_" in m.text


def test_llama31_scaled_rope_engine_graph_matches_eager():
    """Llama-3.1-style model (rope scaling, 128k max positions -> 2048-entry
    block tables in the captured graphs) through the planner: hipGraph replay
    and eager launches agree, and every plan validates."""
    import dataclasses
    from mcp_amd.models.llama import CONFIGS, random_weights
    cfg = dataclasses.replace(CONFIGS["tiny"], name="tiny31", max_pos=131072,
                              rope_scaling=CONFIGS["llama3.1-8b"].rope_scaling)
    model = LlamaModel(cfg, random_weights(cfg, "cuda", seed=5), "cuda")
    reg = MemoryRegistry(synthetic_registry(8, seed=2))
    intents = [synthetic_intent(i) for i in range(6)]
    eager, _ = _plans(model, reg, intents, graphs=False, cascade=False, pipeline=False)
    graph, e2 = _plans(model, reg, intents, graphs=True, cascade=False, pipeline=False)
    assert e2.stats["graph_steps"] > 0 and graph == eager
    names = [s.name for s in reg.list_services()]
    for d in graph:
        validate_dag(d, names)


def test_gqa_padded_group3_model_on_gpu_matches_cpu_and_plans():
    """Llama-3.2-style GQA group 3 padded to 4 (zero pad heads): the GPU
    forward matches the fp32 CPU forward of the same weights, and the planner
    produces valid plans with graph replay == eager."""
    import numpy as np
    from mcp_amd.engine.batch import StepInputs, pack
    from mcp_amd.engine.kv_cache import KVCache
    from mcp_amd.models.llama import LlamaConfig, pad_gqa, random_weights
    pc = pad_gqa(LlamaConfig("g3", hidden=768, layers=2, heads=6, kv_heads=2, ffn=1024,
                             tie_embeddings=True))
    assert pc.group == 4 and pc.group_true == 3
    w = random_weights(pc, "cuda", seed=6, std=0.05)
    model = LlamaModel(pc, w, "cuda")
    T = 100
    ids = torch.randint(0, pc.vocab_size, (T,), generator=torch.Generator().manual_seed(1))
    step = StepInputs(token_ids=ids.int().numpy(), positions=np.arange(T, dtype=np.int32),
                      slots=np.arange(T, dtype=np.int32), q_start=np.asarray([0], np.int32),
                      q_len=np.asarray([T], np.int32), ctx_len=np.asarray([T], np.int32),
                      block_table=np.asarray([[0, 1]], np.int32),
                      logit_rows=np.asarray([T - 1], np.int32))
    kv = KVCache(pc.layers, pc.kv_heads, pc.head_dim, 4, "cuda")
    got = model.forward(pack(step, pc.group, "cuda"), kv).float().cpu()
    import dataclasses
    from mcp_amd.models.llama import LayerWeights, LlamaWeights
    f32 = lambda t: t.float().cpu()
    emb = f32(w.embed)
    wc = LlamaWeights(emb, [LayerWeights(*[f32(getattr(l, fl.name)) for fl in dataclasses.fields(l)])
                            for l in w.layers], f32(w.final_norm), emb)
    kvc = KVCache(pc.layers, pc.kv_heads, pc.head_dim, 4, "cpu", dtype=torch.float32)
    want = LlamaModel(pc, wc, "cpu").forward(pack(step, pc.group, "cpu"), kvc).float()
    assert ((got - want).norm() / want.norm()).item() < 3e-2
    reg = MemoryRegistry(synthetic_registry(8, seed=2))
    intents = [synthetic_intent(i) for i in range(6)]
    eager, _ = _plans(model, reg, intents, graphs=False, cascade=False, pipeline=False)
    graph, e2 = _plans(model, reg, intents, graphs=True, cascade=True, pipeline=False)
    names = [s.name for s in reg.list_services()]
    for d in eager + graph:
        validate_dag(d, names)
    assert e2.stats["graph_steps"] > 0


def test_graph_replay_split_kv_matches_eager(monkeypatch):
    """Split-KV decode attention (K6, forced to 4 splits) inside captured
    hipGraphs: same greedy plans as the eager split path and as no split."""
    model = LlamaModel.random("tiny", "cuda", seed=3)
    reg = MemoryRegistry(synthetic_registry(8, seed=2))
    intents = [synthetic_intent(i) for i in range(4)]
    plain, _ = _plans(model, reg, intents, graphs=False, cascade=False, pipeline=False)
    monkeypatch.setenv("MCP_KV_SPLIT", "4")
    eager, e1 = _plans(model, reg, intents, graphs=False, cascade=False, pipeline=False)
    graph, e2 = _plans(model, reg, intents, graphs=True, cascade=False, pipeline=False)
    assert e1.stats["kv_split_steps"] > 0 and e2.stats["graph_split_steps"] > 0
    assert graph == eager
    same = sum(x == y for x, y in zip(plain, eager))
    assert same >= len(plain) - 1, same


def test_llama3_8b_full_width_layers_match_fp32():
    """Two Llama-3-8B decoder layers at full width (H 4096, 32 q / 8 kv heads,
    FFN 14336, vocab 128256) on the HIP kernels vs the fp32 CPU forward of the
    same weights: a 300-token prefill (AGPR / split-K GEMMs, fused QKV+RoPE
    epilogue, SwiGLU epilogue, 4-wave attention items) and then a ragged
    decode + jump-forward step over the cached KV (1-wave items, small-M
    GEMM paths)."""
    import dataclasses
    import numpy as np
    from mcp_amd.engine.batch import StepInputs, pack
    from mcp_amd.engine.kv_cache import KVCache
    from mcp_amd.models.llama import CONFIGS, LayerWeights, LlamaWeights, random_weights
    cfg = dataclasses.replace(CONFIGS["llama3-8b"], name="8b-2layer", layers=2)
    w = random_weights(cfg, "cuda", seed=11, std=0.02)
    g = torch.Generator(device="cuda").manual_seed(4)
    for lw in w.layers:                  # non-trivial RMSNorm weights (folded by the GPU model)
        lw.attn_norm.copy_(1 + 0.2 * torch.randn(lw.attn_norm.shape, device="cuda", generator=g))
        lw.mlp_norm.copy_(1 + 0.2 * torch.randn(lw.mlp_norm.shape, device="cuda", generator=g))
    f32 = lambda t: t.float().cpu()
    wc = LlamaWeights(f32(w.embed), [LayerWeights(*[f32(getattr(l, fl.name)) for fl in dataclasses.fields(l)])
                                     for l in w.layers], f32(w.final_norm), f32(w.lm_head))
    model = LlamaModel(cfg, w, "cuda")             # fused-norm forward (TP = 1)
    assert model.fused_norm
    import os
    os.environ["MCP_FUSED_NORM"] = "0"             # the fp32 reference: standalone RMSNorm
    try:
        cpu = LlamaModel(cfg, wc, "cpu")
    finally:
        del os.environ["MCP_FUSED_NORM"]
    assert not cpu.fused_norm
    nb = 16
    kv = KVCache(cfg.layers, cfg.kv_heads, cfg.head_dim, nb, "cuda")
    kvc = KVCache(cfg.layers, cfg.kv_heads, cfg.head_dim, nb, "cpu", dtype=torch.float32)
    rng = np.random.default_rng(3)
    T = 300                                      # prefill: 5 blocks
    step = StepInputs(token_ids=rng.integers(0, cfg.vocab_size, T).astype(np.int32),
                      positions=np.arange(T, dtype=np.int32), slots=np.arange(T, dtype=np.int32),
                      q_start=np.asarray([0], np.int32), q_len=np.asarray([T], np.int32),
                      ctx_len=np.asarray([T], np.int32),
                      block_table=np.asarray([[0, 1, 2, 3, 4, 5]], np.int32),
                      logit_rows=np.asarray([T - 1, 100], np.int32))
    got = model.forward(pack(step, cfg.group, "cuda"), kv).float().cpu()
    want = cpu.forward(pack(step, cfg.group, "cpu"), kvc).float()
    assert ((got - want).norm() / want.norm()).item() < 3e-2
    # ragged follow-up step on the cached prefix: the same sequence decodes 1
    # token, a second one (own blocks 8-9) prefills a 7-token span
    ids = rng.integers(0, cfg.vocab_size, 8).astype(np.int32)
    step2 = StepInputs(token_ids=ids, positions=np.asarray([T] + list(range(7)), np.int32),
                       slots=np.asarray([T] + [8 * 64 + i for i in range(7)], np.int32),
                       q_start=np.asarray([0, 1], np.int32), q_len=np.asarray([1, 7], np.int32),
                       ctx_len=np.asarray([T + 1, 7], np.int32),
                       block_table=np.asarray([[0, 1, 2, 3, 4, 5], [8, 9, 0, 0, 0, 0]], np.int32),
                       logit_rows=np.asarray([0, 7], np.int32))
    got2 = model.forward(pack(step2, cfg.group, "cuda"), kv).float().cpu()
    want2 = cpu.forward(pack(step2, cfg.group, "cpu"), kvc).float()
    assert ((got2 - want2).norm() / want2.norm()).item() < 3e-2


def test_weight_prefetch_step_with_no_logit_rows_joins_side_stream(monkeypatch):
    """with MCP_WEIGHT_PREFETCH on, a step that samples no row
    (the last layer returns early) still joins the prefetch side stream:
    eagerly, and inside a captured hipGraph (an unjoined side stream is a
    capture error)."""
    import numpy as np
    import mcp_amd.models.llama as llama_mod
    from mcp_amd.engine.batch import StepInputs, pack
    from mcp_amd.engine.kv_cache import KVCache
    monkeypatch.setattr(llama_mod, "_PF_ON", True)
    model = LlamaModel.random("tiny", "cuda", seed=3)
    assert model._pf_side is not None and model.fused_norm
    cfg = model.cfg
    T = 8
    step = StepInputs(token_ids=np.arange(T, dtype=np.int32), positions=np.arange(T, dtype=np.int32),
                      slots=np.arange(T, dtype=np.int32), q_start=np.asarray([0], np.int32),
                      q_len=np.asarray([T], np.int32), ctx_len=np.asarray([T], np.int32),
                      block_table=np.asarray([[0]], np.int32),
                      logit_rows=np.zeros(0, np.int32))
    kv = KVCache(cfg.layers, cfg.kv_heads, cfg.head_dim, 4, "cuda")
    packed = pack(step, cfg.group, "cuda")
    out = model.forward(packed, kv)
    assert out.shape[0] == 0
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            out = model.forward(packed, kv)
    g.replay()
    torch.cuda.synchronize()
    assert out.shape[0] == 0
