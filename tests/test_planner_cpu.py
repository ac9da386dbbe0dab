"""Planner tests on CPU: grammar, engine plumbing with the tiny
Llama config through the fp32 reference ops, API wiring of the local planner."""
import asyncio
import json
import random
import re

import httpx
import numpy as np
import time

import pytest
import torch
from fastapi.testclient import TestClient

from mcp_amd.api.server import create_app
from mcp_amd.config import Settings
from mcp_amd.engine.batch import build_work
from mcp_amd.engine.engine import LLMEngine
from mcp_amd.engine.kv_cache import BlockAllocator
from mcp_amd.models.llama import LlamaModel
from mcp_amd.orchestrator import validate_dag
from mcp_amd.planner.grammar import DagDecoder, GrammarSpec, build_trie
from mcp_amd.planner.local import LocalPlanner
from mcp_amd.planner.prompt import synthetic_intent
from mcp_amd.planner.tokenizer import get_tokenizer
from mcp_amd.registry import MemoryRegistry, make_service, synthetic_registry
from mcp_amd.retrieval.store import SchemaIndex, hash_embed


def random_walk(spec, rng):
    dec = DagDecoder(spec)
    toks = dec.advance()
    n = 0
    while not dec.done:
        allowed = dec.allowed()
        assert len(allowed) >= 2
        dec.feed(rng.choice(allowed))
        toks += dec.advance()
        n += 1
    return dec, toks, n


def model_view(text: str, by) -> str:
    """The compact model view of an emitted DAG (planner/grammar.py): no
    endpoints; of the edges only those whose target has a registry fallback,
    as {"to":...} with the fallback mark the model chose."""
    head, edges = re.sub(r',"endpoint":"[^"]*"', "", text).split('],"edges":[')
    parts = []
    for e in json.loads("[" + edges[:-2] + "]"):
        if by[e["to"]]["fallback"]:
            parts.append('{"to":' + json.dumps(e["to"]) +
                         (',"fallback":true}' if "fallback" in e else "}"))
    return head + '],"edges":[' + "".join(parts) + "]}"


@pytest.mark.parametrize("compact", [False, True])
@pytest.mark.parametrize("nsvc,max_nodes", [(1, 3), (3, 6), (10, 6), (50, 8)])
def test_grammar_always_valid_t2(nsvc, max_nodes, compact):
    tok = get_tokenizer()
    reg = synthetic_registry(nsvc, seed=nsvc)
    spec = GrammarSpec(reg, tok, max_nodes=max_nodes, compact=compact)
    rng = random.Random(0)
    for _ in range(40):
        dec, toks, n = random_walk(spec, rng)
        dag = dec.result()
        validate_dag(dag, [s["name"] for s in reg])
        assert len(dag["nodes"]) <= max_nodes
        # the token stream decodes to exactly the emitted JSON text (compact:
        # to its model view, URLs left to the registry)
        by = {s["name"]: s for s in reg}
        assert tok.decode(toks) == (model_view(dec.text, by) if compact else dec.text)
        for node in dag["nodes"]:
            assert node["endpoint"] == by[node["name"]]["endpoint"]
            assert set(node["inputs"]) == set(by[node["name"]].input_keys())
        for e in dag["edges"]:
            if "fallback" in e:
                assert e["fallback"] == by[e["to"]]["fallback"]


def test_trie_prefix_free_check():
    with pytest.raises(ValueError):
        build_trie([[1, 2], [1, 2, 3]])
    t = build_trie([[1, 2], [1, 3], [4]])
    assert sorted(t.children) == [1, 4]


def test_block_allocator_refcounts():
    a = BlockAllocator(8)
    b = a.alloc(3)
    a.incref(b[:2])
    a.free(b)
    assert a.num_free == 6
    a.free(b[:2])
    assert a.num_free == 8
    with pytest.raises(RuntimeError):
        a.free(b[:1])


def test_work_split():
    w = build_work([1, 3, 40, 0, 17], group=4)
    assert w[1] == ([0, 1], [0, 0])
    assert w[4][0] == [2, 2, 2, 4, 4]
    assert w[4][1] == [0, 16, 32, 0, 16]


@pytest.fixture(scope="module")
def tiny_engine():
    torch.manual_seed(0)
    model = LlamaModel.random("tiny", "cpu", seed=1)
    return LLMEngine(model, num_blocks=256, max_batch=16, max_step_tokens=4096)


def test_engine_plans_valid_dags(tiny_engine):
    reg = MemoryRegistry(synthetic_registry(5, seed=2))
    planner = LocalPlanner(tiny_engine, reg, max_nodes=4)
    intents = [synthetic_intent(i) for i in range(3)]
    dags = planner.plan_many(intents)
    assert len(dags) == 3
    for d in dags:
        validate_dag(d, [s.name for s in reg.list_services()])
    assert tiny_engine.alloc.num_free == tiny_engine.kv.num_blocks     # every block returned
    # greedy decoding is deterministic across runs
    tiny_engine.temperature = 0.0
    a = planner.plan_many(intents[:2])
    b = planner.plan_many(intents[:2])
    tiny_engine.temperature = 0.2
    assert a == b


def test_prefix_sharing_matches_unshared(tiny_engine):
    """A request decoded on shared prefix blocks equals the same request decoded alone."""
    reg = MemoryRegistry(synthetic_registry(6, seed=3))
    planner = LocalPlanner(tiny_engine, reg, max_nodes=3)
    tiny_engine.temperature = 0.0
    try:
        together = planner.plan_many([synthetic_intent(1), synthetic_intent(2)])
        alone = planner.plan_many([synthetic_intent(2)])
    finally:
        tiny_engine.temperature = 0.2
    assert together[1] == alone[0]


def test_local_planner_behind_api(tiny_engine):
    reg = MemoryRegistry(synthetic_registry(4, seed=5))
    planner = LocalPlanner(tiny_engine, reg, max_nodes=3)

    def h(request):
        return httpx.Response(200, json={"ok": True})
    app = create_app(Settings(), registry=reg, planner=planner, transport=httpx.MockTransport(h))
    with TestClient(app) as c:
        r = c.post("/plan", json={"intent": "charge the order and email the receipt"})
        assert r.status_code == 200
        validate_dag(r.json()["graph"], [s.name for s in reg.list_services()])
        r2 = c.post("/plan_and_execute", json={"intent": "score the order"})
        assert r2.status_code == 200 and set(r2.json()) == {"results", "errors"}
        # per-request phases reach /metrics
        text = c.get("/metrics").text
        for phase in ("retrieval_s", "prompt_s", "queue_s", "ttft_s", "decode_s", "parse_s",
                      "execute_latency_s"):
            assert f"mcp_{phase}" in text, phase


def test_retrieval_cpu_prunes_prompt():
    reg = MemoryRegistry(synthetic_registry(300, seed=7))
    idx = SchemaIndex(reg, dim=512, device="cpu")
    svcs = reg.list_services()
    got = idx.search("payment charge amount currency", 8, svcs)
    assert len(got) == 8
    assert any("payment" in s.name or "charge" in s.name for s in got)
    e = hash_embed(["a b c", "a b c"], 64)
    assert np.allclose(e[0], e[1]) and abs(np.linalg.norm(e[0]) - 1) < 1e-5


def _shared_block_fraction(planner, intents, svcs):
    """Replay of the prompts' 64-token block chains (the engine's block-level
    prefix cache keys): the fraction of blocks an earlier prompt computed."""
    from mcp_amd.planner.prompt import build_prompt_parts
    seen, hit, tot = set(), 0, 0
    for it in intents:
        prefix, _ = build_prompt_parts(planner.candidates(it, svcs), it, compact=True)
        t = planner.tok.prompt_ids(prefix)
        h = ()
        for b in range(len(t) // 64):
            h = hash((h, tuple(t[b * 64:(b + 1) * 64])))
            tot += 1
            hit += h in seen
            seen.add(h)
    return hit / tot


def test_retrieval_popularity_order_shares_more_prefix_blocks(monkeypatch):
    """MCP_RETRIEVAL_ORDER=popular (default): the same retrieved sets, ordered
    most-retrieved first, share more prompt-prefix blocks than name or score
    order; the order is a permutation of the retrieved set and is stable
    between rank snapshots."""
    reg = MemoryRegistry(synthetic_registry(2000, seed=3))
    svcs = reg.list_services()
    idx = SchemaIndex(reg, dim=512, device="cpu")
    idx.refresh()
    intents = [synthetic_intent(i) for i in range(96)]
    frac = {}
    for order in ("popular", "name", "score"):
        monkeypatch.setattr(LocalPlanner, "ORDER", order)
        pl = LocalPlanner(None, reg, retriever=idx, retrieval_threshold=48, topk=32)
        frac[order] = _shared_block_fraction(pl, intents, svcs)
    assert frac["popular"] > frac["name"] > frac["score"], frac
    monkeypatch.setattr(LocalPlanner, "ORDER", "popular")
    pl = LocalPlanner(None, reg, retriever=idx, retrieval_threshold=48, topk=32)
    for it in intents[:70]:                      # snapshots at 16 and 64 requests
        pl.candidates(it, svcs)
    a = pl.candidates(intents[3], svcs)
    b = pl.candidates(intents[3], svcs)          # no snapshot in between: same order
    assert [s["name"] for s in a] == [s["name"] for s in b]
    assert sorted(s["name"] for s in a) == sorted(s["name"] for s in idx.search(intents[3], 32, svcs))


def test_gate_up_interleave_roundtrip():
    from mcp_amd.ops import reference as ref
    g, u = torch.randn(64, 8), torch.randn(64, 8)
    w = ref.interleave_gate_up(g, u)
    g2, u2 = ref.deinterleave_gate_up(w)
    assert torch.equal(g, g2) and torch.equal(u, u2)
    X = torch.randn(3, 8)
    assert torch.allclose(ref.gemm_silu(X, w), torch.nn.functional.silu(X @ g.t()) * (X @ u.t()), atol=1e-5)


def test_pipelined_engine_matches_synchronous():
    """Two launch cohorts in flight (host updates one while the device runs the
    other) produce the same greedy plans as the synchronous engine."""
    reg = MemoryRegistry(synthetic_registry(6, seed=4))
    intents = [synthetic_intent(i) for i in range(5)]
    out = []
    for pipe in (False, True):
        torch.manual_seed(0)
        model = LlamaModel.random("tiny", "cpu", seed=1)
        eng = LLMEngine(model, num_blocks=256, max_batch=16, temperature=0.0, pipeline=pipe)
        planner = LocalPlanner(eng, reg, max_nodes=3)
        out.append(planner.plan_many(intents))
        assert eng.alloc.num_free == eng.kv.num_blocks and not eng.inflight
    assert out[0] == out[1]


@pytest.mark.parametrize("temperature", [0.0, 0.2])
def test_lookahead_engine_matches_synchronous(temperature, monkeypatch):
    """Decision lookahead (the next step launched over every outcome of the
    pending choices, the sampled outcome picked on the device side by
    ops.branch_select) produces the same plans as the synchronous engine, one
    intent at a time and several at once; every KV block comes back."""
    from mcp_amd.engine import native
    if not native.available():
        pytest.skip("native runtime not built")
    reg = MemoryRegistry(synthetic_registry(7, seed=4))
    intents = [synthetic_intent(i) for i in range(4)]
    out, stats = [], []
    import itertools
    from mcp_amd.engine import engine as engine_mod
    for look in (False, True):
        torch.manual_seed(0)
        # the sampling counter is (request uid, sample index): same uids in both runs
        monkeypatch.setattr(engine_mod, "_uid", itertools.count(1))
        model = LlamaModel.random("tiny", "cpu", seed=1)
        eng = LLMEngine(model, num_blocks=256, max_batch=16, temperature=temperature,
                        lookahead=look)
        planner = LocalPlanner(eng, reg, max_nodes=4, min_nodes=2)
        res = [planner.plan_many([it])[0] for it in intents[:2]]
        res += planner.plan_many(intents)
        out.append(res)
        stats.append(dict(eng.stats))
        assert eng.alloc.num_free == eng.kv.num_blocks and not eng._look and not eng.inflight
    assert out[0] == out[1]
    assert stats[0]["lookahead_steps"] == 0 and stats[1]["lookahead_steps"] > 0
    assert stats[0]["samples"] == stats[1]["samples"]


@pytest.mark.parametrize("temperature", [0.0, 0.2])
def test_lookahead_admits_arrivals_and_matches_synchronous(temperature, monkeypatch):
    """Requests arriving while the engine is in decision lookahead join the
    next lookahead step (their prompt tokens after the lookahead rows,
    MCP_LOOKAHEAD_ADMIT) and every plan equals the synchronous engine's under
    the same arrival schedule."""
    from mcp_amd.engine import native
    if not native.available():
        pytest.skip("native runtime not built")
    import itertools
    from mcp_amd.engine import engine as engine_mod
    reg = MemoryRegistry(synthetic_registry(7, seed=4))
    out, stats = [], []
    for look in (False, True):
        torch.manual_seed(0)
        monkeypatch.setattr(engine_mod, "_uid", itertools.count(1))
        model = LlamaModel.random("tiny", "cpu", seed=1)
        eng = LLMEngine(model, num_blocks=256, max_batch=16, temperature=temperature,
                        lookahead=look)
        planner = LocalPlanner(eng, reg, max_nodes=4, min_nodes=2)
        planner.plan_many([synthetic_intent(99)])           # the registry prefix is computed
        seqs, k = [], 0
        for i in range(4):
            dec, ptoks, stoks = planner.prepare(synthetic_intent(i))
            seqs.append(eng.submit(dec, stoks, prefix_tokens=ptoks))
            for _ in range(3 + i):                          # arrivals mid-decode
                if eng.has_work():
                    eng.step()
                    k += bool(eng._look)
        eng.run()
        out.append([q.result for q in seqs])
        stats.append((dict(eng.stats), k))
        assert all(q.error is None for q in seqs)
        assert not eng._look and not eng.running
    assert out[0] == out[1]
    assert stats[1][0]["lookahead_steps"] > 0 and stats[1][1] > 0
    assert stats[1][0]["lookahead_admitted"] > 0, stats[1][0]


def test_lookahead_hold_pumps_arrivals_into_branch_step(monkeypatch):
    """The lookahead hold (MCP_LOOKAHEAD_HOLD): once a step time is measured,
    the branch launch waits until shortly before the current step's end and
    pumps the driver's arrivals meanwhile; an arrival ends the wait and joins
    the branch step.  On the CPU the forward is synchronous, so the sampled-
    token wait is slowed to look device-bound."""
    from mcp_amd.engine import native
    if not native.available():
        pytest.skip("native runtime not built")
    from mcp_amd.engine import engine as engine_mod
    reg = MemoryRegistry(synthetic_registry(7, seed=4))
    torch.manual_seed(0)
    model = LlamaModel.random("tiny", "cpu", seed=1)
    eng = LLMEngine(model, num_blocks=256, max_batch=16, temperature=0.0, lookahead=True)
    planner = LocalPlanner(eng, reg, max_nodes=4, min_nodes=2)
    planner.plan_many([synthetic_intent(99)])           # the registry prefix is computed
    real_wait = engine_mod.LLMEngine._wait_tokens

    def slow_wait(self, L):
        time.sleep(0.004)                                # the device "runs" for 4 ms
        return real_wait(self, L)
    monkeypatch.setattr(engine_mod.LLMEngine, "_wait_tokens", slow_wait)
    monkeypatch.setattr(engine_mod.LLMEngine, "LOOK_LEAD_S", 0.001)
    pending = [planner.prepare(synthetic_intent(i)) for i in range(1, 4)]
    seqs, calls = [], []

    def pump():
        calls.append(len(eng._look))
        if len(calls) % 3 == 0 and pending:             # an arrival during some holds
            dec, ptoks, stoks = pending.pop(0)
            seqs.append(eng.submit(dec, stoks, prefix_tokens=ptoks))
            return 1
        return 0
    eng.poll_arrivals = pump
    dec, ptoks, stoks = planner.prepare(synthetic_intent(0))
    seqs.append(eng.submit(dec, stoks, prefix_tokens=ptoks))
    eng.run()
    while pending:                                       # arrivals the run did not pump
        dec, ptoks, stoks = pending.pop(0)
        seqs.append(eng.submit(dec, stoks, prefix_tokens=ptoks))
        eng.run()
    assert calls, "the hold never pumped arrivals"
    assert eng.stats.get("look_hold_s", 0.0) > 0.0
    assert eng.stats["lookahead_admitted"] > 0, eng.stats
    assert all(q.error is None and q.result for q in seqs)
    eng.drop_prefixes()                                  # the cached registry prefix
    assert not eng._look and not eng.running and eng.alloc.num_free == eng.kv.num_blocks


def test_graph_static_layout_matches_dynamic():
    """The fixed per-bucket layout used by captured hipGraphs (padding tokens,
    empty dummy sequences, padded work lists and allowed sets) computes the same
    hidden states and samples as the dynamic layout (CPU reference ops)."""
    from mcp_amd import ops
    from mcp_amd.engine.batch import StepInputs, pack, views
    from mcp_amd.engine.graphs import GraphRunner
    torch.manual_seed(0)
    model = LlamaModel.random("tiny", "cpu", seed=2)
    eng = LLMEngine(model, num_blocks=64, max_batch=8, temperature=0.0, graphs=False)
    gr = GraphRunner(model, eng.kv, 0.0, 0)
    rng = np.random.default_rng(0)
    q_lens, ctx = [3, 1, 9], [3, 40, 9]
    T = sum(q_lens)
    blocks = [[0], [1], [2]]
    ids = rng.integers(0, 1000, T).astype(np.int32)
    pos = np.concatenate([np.arange(c - q, c) for q, c in zip(q_lens, ctx)]).astype(np.int32)
    slots = np.concatenate([np.asarray(b)[p // 64] * 64 + p % 64 for b, p in
                            zip(blocks, np.split(pos, np.cumsum(q_lens)[:-1]))]).astype(np.int32)
    qs = np.concatenate([[0], np.cumsum(q_lens)[:-1]]).astype(np.int32)
    rows = (qs + np.asarray(q_lens) - 1).astype(np.int32)
    allowed = [[5, 9, 11], [7, 8], [1, 2, 3, 4]]
    ptr = np.concatenate([[0], np.cumsum([len(a) for a in allowed])]).astype(np.int32)
    step = StepInputs(token_ids=ids, positions=pos, slots=slots, q_start=qs,
                      q_len=np.asarray(q_lens, np.int32), ctx_len=np.asarray(ctx, np.int32),
                      block_table=np.asarray(blocks, np.int32), logit_rows=rows,
                      allow_ptr=ptr, allow_ids=np.concatenate(allowed).astype(np.int32),
                      sample_ctr=np.asarray([1, 2, 3], np.int32))
    # make the cached context (positions before the new tokens) deterministic
    eng.kv.data.normal_()
    kv0 = eng.kv.data.clone()
    d = pack(step, model.cfg.group, "cpu")
    h_dyn = model.forward(d, eng.kv)
    t_dyn = ops.sample_allowed(h_dyn, model.w.lm_head, d.allow_ptr, d.allow_ids, d.sample_ctr, 0.0, 0)
    eng.kv.data.copy_(kv0)
    b, sb = gr.bucket_for(step)
    assert (b, sb) == (16, 8)
    host = gr.pack_static(step, b, sb=sb)
    ds = views(torch.from_numpy(host), gr._sizes(b, sb=sb) + [gr._caps(b, sb)[0], 0])[0]
    h_st = model.forward(ds, eng.kv)
    t_st = ops.sample_allowed(h_st, model.w.lm_head, ds.allow_ptr, ds.allow_ids, ds.sample_ctr, 0.0, 0)
    assert torch.allclose(h_st[:3].float(), h_dyn.float(), atol=1e-5)
    assert t_st[:3].tolist() == t_dyn.tolist()
    assert (t_st[3:] == -1).all()          # padded rows have empty allowed sets
    # the narrow block-table width class + a padded copy-on-write list: the
    # real pair is copied, the (-1, -1) padding is skipped, same forward
    eng.kv.data.copy_(kv0)
    w = gr.width_for(int(step.block_table.shape[1]))
    assert w == 32
    host = gr.pack_static(step, b, w, [(5, 6)], sb)
    ds, csrc, cdst = views(torch.from_numpy(host), gr._sizes(b, w, sb) + [gr._caps(b, sb)[0], 0])
    assert csrc.numel() == gr._ncopy(b, sb) and (csrc[1:] == -1).all()
    ops.copy_blocks(eng.kv.data, csrc, cdst)
    assert torch.equal(eng.kv.data[:, :, 6], kv0[:, :, 5])
    assert torch.equal(eng.kv.data[:, :, 7:], kv0[:, :, 7:])
    h_w = model.forward(ds, eng.kv)
    assert torch.allclose(h_w[:3].float(), h_dyn.float(), atol=1e-5)


def test_graph_static_layout_carries_cascade_sizes():
    """hipGraph layouts carry the cascade prefix on the device: segment 15 =
    [pre_tokens, pre_keys, prefix blocks...] (views() with pre_tokens -1 turns
    it into AttnMeta.pre_dims / pre_bt), kv_begin per sequence, and a step
    without cascade packs pre_tokens 0 (the prefix pass then exits at once)."""
    from mcp_amd.engine.batch import StepInputs, views
    from mcp_amd.engine.graphs import GraphRunner
    model = LlamaModel.random("tiny", "cpu", seed=2)
    eng = LLMEngine(model, num_blocks=64, max_batch=8, temperature=0.0, graphs=False)
    gr = GraphRunner(model, eng.kv, 0.0, 0)
    q_lens, ctx = [2, 3], [130, 140]
    T = sum(q_lens)
    step = StepInputs(token_ids=np.arange(T, dtype=np.int32),
                      positions=np.asarray([128, 129, 137, 138, 139], np.int32),
                      slots=np.asarray([3 * 64, 3 * 64 + 1, 4 * 64 + 9, 4 * 64 + 10, 4 * 64 + 11], np.int32),
                      q_start=np.asarray([0, 2], np.int32), q_len=np.asarray(q_lens, np.int32),
                      ctx_len=np.asarray(ctx, np.int32),
                      block_table=np.asarray([[0, 1, 3], [0, 1, 4]], np.int32),
                      logit_rows=np.asarray([1, 4], np.int32),
                      allow_ptr=np.asarray([0, 2, 4], np.int32),
                      allow_ids=np.asarray([5, 6, 7, 8], np.int32),
                      sample_ctr=np.asarray([1, 2], np.int32))
    step.kv_begin = np.asarray([128, 128], np.int32)
    step.pre_bt = np.asarray([0, 1], np.int32)
    step.pre_tokens = T
    b, sb = gr.bucket_for(step)
    w = gr.width_for(3)
    host = gr.pack_static(step, b, w, sb=sb)
    d = views(torch.from_numpy(host), gr._sizes(b, w, sb) + [gr._caps(b, sb)[0], -1, 1])[0]
    m = d.attn
    assert m.pre_dims.tolist() == [T, 128]
    assert m.pre_bt[:2].tolist() == [0, 1] and m.pre_bt.numel() == w
    assert m.kv_begin[:2].tolist() == [128, 128] and int(m.kv_begin[2:].abs().sum()) == 0
    assert m.pre_tokens == b and m.pre_keys == w * 64          # grid capacities
    step.pre_tokens, step.pre_bt, step.kv_begin = 0, None, None
    d2 = views(torch.from_numpy(gr.pack_static(step, b, w, sb=sb)),
               gr._sizes(b, w, sb) + [gr._caps(b, sb)[0], -1, 1])[0]
    assert d2.attn.pre_dims.tolist() == [0, 0] and int(d2.attn.kv_begin.abs().sum()) == 0


def test_engine_stall_watchdog_returns_503():
    """A step that stops making progress (hung GPU) fails pending requests with
    EngineStalled -> HTTP 503, and /healthz reports the replica unhealthy."""
    import time as _time
    model = LlamaModel.random("tiny", "cpu", seed=1)
    eng = LLMEngine(model, num_blocks=128, max_batch=4)
    reg = MemoryRegistry(synthetic_registry(3, seed=5))
    planner = LocalPlanner(eng, reg, max_nodes=2, watchdog_s=0.3)
    real_step = eng.step

    def hung_step():
        _time.sleep(1.5)
        return real_step()
    eng.step = hung_step

    def h(request):
        return httpx.Response(200, json={})
    app = create_app(Settings(), registry=reg, planner=planner, transport=httpx.MockTransport(h))
    with TestClient(app) as c:
        r = c.post("/plan", json={"intent": "charge the order"})
        assert r.status_code == 503
        assert c.get("/healthz").status_code == 503
    planner._stop.set()


def test_engine_stall_recovers_after_the_step_returns():
    """Stall recovery: the hung step's requests fail with 503, and once the
    step returns the planner aborts what the engine still holds (blocks back
    to the allocator) and serves new requests again - not 503 forever."""
    import time as _time
    model = LlamaModel.random("tiny", "cpu", seed=1)
    eng = LLMEngine(model, num_blocks=128, max_batch=4)
    reg = MemoryRegistry(synthetic_registry(3, seed=5))
    planner = LocalPlanner(eng, reg, max_nodes=2, watchdog_s=0.3)
    real_step = eng.step
    hang = {"left": 1}

    def step_once_hung():
        if hang["left"]:
            hang["left"] -= 1
            _time.sleep(1.5)
        return real_step()
    eng.step = step_once_hung
    free0 = eng.alloc.num_free

    def h(request):
        return httpx.Response(200, json={})
    app = create_app(Settings(), registry=reg, planner=planner, transport=httpx.MockTransport(h))
    names = [s.name for s in reg.list_services()]
    with TestClient(app) as c:
        assert c.post("/plan", json={"intent": "charge the order"}).status_code == 503
        t0 = _time.time()
        while planner.stalled and _time.time() - t0 < 30:
            _time.sleep(0.05)
        assert not planner.stalled
        r = c.post("/plan", json={"intent": "refund the order"})
        assert r.status_code == 200, r.text
        validate_dag(r.json()["graph"], names)
        assert c.get("/healthz").status_code == 200
    planner._stop.set()
    assert not eng.has_work()
    if free0 is not None:
        eng.drop_prefixes()                 # the cached registry prefix is the only holder left
        assert eng.alloc.num_free == free0


def test_kv_split_rule():
    """Split-KV only for decode-sized items that underfill the chip with own
    key ranges of >= 4 tiles; >= 4 tiles per split from 32 tiles, >= 2 below
    (a single intent's ~700-key context; 1 below 16 tiles for spans of <= 8
    rows with MCP_KV_SPLIT_SHORT=1); forced / disabled by MCP_KV_SPLIT."""
    from mcp_amd.engine.batch import choose_kv_splits
    assert choose_kv_splits([1], [32768], 4, 8) == 64          # batch-1 decode, 32k keys
    assert choose_kv_splits([1] * 4, [32768] * 4, 4, 8) == 16
    assert choose_kv_splits([1], [700], 4, 8) == 4               # single intent: 11 tiles / 2 -> 5 -> power of two
    assert choose_kv_splits([1], [400], 4, 8) == 2               # 7 tiles: 2 splits (serving-size steps)
    # MCP_KV_SPLIT_SHORT=1 (opt-in, round 6): short contexts with decode-sized
    # spans split down to one tile per split
    os_env = __import__("os").environ
    os_env["MCP_KV_SPLIT_SHORT"] = "1"
    import importlib
    import mcp_amd.engine.batch as batch_mod
    try:
        importlib.reload(batch_mod)
        assert batch_mod.choose_kv_splits([1], [700], 4, 8) == 8    # 11 tiles -> 8
        assert batch_mod.choose_kv_splits([1], [400], 4, 8) == 4    # 7 tiles -> 4
        assert batch_mod.choose_kv_splits([16], [700], 4, 8) == 4   # 16-row span: 11 / 2 -> 4
    finally:
        del os_env["MCP_KV_SPLIT_SHORT"]
        importlib.reload(batch_mod)
    assert choose_kv_splits([1], [150], 4, 8) == 1               # < 4 tiles: unsplit
    assert choose_kv_splits([1] * 64, [8192] * 64, 4, 8) == 1    # 512 items already fill it
    assert choose_kv_splits([300], [32768], 4, 8) == 4           # 19 4-wave items: underfilled
    assert choose_kv_splits([3000], [32768], 4, 8) == 1          # a big prefill fills the chip
    assert choose_kv_splits([1], [2048], 4, 8) == 8              # 32 tiles -> 8 splits of 4
    import os
    os.environ["MCP_KV_SPLIT"] = "0"
    try:
        assert choose_kv_splits([1], [32768], 4, 8) == 1
    finally:
        del os.environ["MCP_KV_SPLIT"]


def test_prefix_split_rule(monkeypatch):
    """Cascade prefix key split: only small grids (<= a quarter of the CUs)
    split; 0 disables; N forces N (bounded by the tile count)."""
    from mcp_amd import ops
    monkeypatch.delenv("MCP_PREFIX_SPLIT", raising=False)
    assert ops.prefix_splits(16, 704, 8) == 5          # 8 workgroups, 11 tiles
    assert ops.prefix_splits(192, 704, 8) == 5         # 48 workgroups
    assert ops.prefix_splits(256, 704, 8) == 5         # 64 = 256 / 4
    assert ops.prefix_splits(288, 704, 8) == 1         # 72 > 64: no split
    assert ops.prefix_splits(16, 128, 8) == 1          # 2 tiles: nothing to split
    monkeypatch.setenv("MCP_PREFIX_SPLIT", "0")
    assert ops.prefix_splits(16, 704, 8) == 1
    monkeypatch.setenv("MCP_PREFIX_SPLIT", "3")
    assert ops.prefix_splits(4096, 704, 8) == 3


def test_launch_ahead_matches_plain_submit():
    """submit_many(launch_ahead=True) launches the batch's prefix job before the
    suffixes are tokenised and retires it in the next step: same greedy plans,
    all blocks returned, nothing left in flight; a second launch_ahead while a
    step is in flight does nothing."""
    reg = MemoryRegistry(synthetic_registry(6, seed=4))
    intents = [synthetic_intent(i) for i in range(5)]
    out = []
    for ahead in (False, True):
        torch.manual_seed(0)
        model = LlamaModel.random("tiny", "cpu", seed=1)
        eng = LLMEngine(model, num_blocks=256, max_batch=16, temperature=0.0, graphs=False)
        planner = LocalPlanner(eng, reg, max_nodes=3)
        seqs = planner.submit_many(intents, launch_ahead=ahead)
        assert bool(eng.inflight) == ahead
        if ahead:
            assert not eng.launch_ahead()              # a step is already in flight
        eng.run()
        assert eng.alloc.num_free == eng.kv.num_blocks and not eng.inflight
        out.append([s.result for s in seqs])
    assert out[0] == out[1]


def test_context_exhaustion_fails_the_request():
    """A plan that would run past the model's max_pos fails with a clear error
    (no step is ever issued at positions beyond the RoPE table), the blocks go
    back to the allocator and the engine keeps serving."""
    import dataclasses
    from mcp_amd.models.llama import get_config, random_weights
    reg = MemoryRegistry(synthetic_registry(4, seed=3))
    cfg = get_config("tiny")
    probe = LocalPlanner(LLMEngine(LlamaModel(cfg, random_weights(cfg, "cpu", seed=1), "cpu"),
                                   num_blocks=64, max_batch=4, graphs=False), reg, max_nodes=3)
    _, ptoks, stoks = probe.prepare("charge the order")
    n_prompt = len(ptoks) + len(stoks)
    small = dataclasses.replace(cfg, max_pos=n_prompt + 6)
    eng = LLMEngine(LlamaModel(small, random_weights(small, "cpu", seed=1), "cpu"),
                    num_blocks=64, max_batch=4, temperature=0.0, graphs=False)
    seen = []
    real_step = eng.step

    def step():
        for s in eng.running:
            seen.append(s.num_cached + len(s.pending))
        return real_step()
    eng.step = step
    planner = LocalPlanner(eng, reg, max_nodes=3)
    free0 = eng.alloc.num_free
    with pytest.raises(RuntimeError, match="context exhausted"):
        planner.plan_many(["charge the order"])
    assert max(seen) <= small.max_pos
    assert eng.alloc.num_free == free0 and not eng.running
    planner._stop.set()


def test_prefix_cache_yields_blocks_when_the_pool_is_full():
    """With retrieval every request brings its own registry prefix; cached
    prefixes must give their blocks back when the pool runs dry instead of
    failing the request with OutOfBlocks."""
    from mcp_amd.retrieval.store import SchemaIndex
    model = LlamaModel.random("tiny", "cpu", seed=1)
    eng = LLMEngine(model, num_blocks=24, max_batch=4, temperature=0.0, graphs=False)
    reg = MemoryRegistry(synthetic_registry(60, seed=7))
    retr = SchemaIndex(reg, dim=64, device="cpu")
    retr.refresh()
    planner = LocalPlanner(eng, reg, max_nodes=2, retriever=retr, retrieval_threshold=8, topk=4)
    names = [s.name for s in reg.list_services()]
    intents = [synthetic_intent(100 + i) for i in range(8)]
    prefix_blocks = sum(len(planner.prepare(x)[1]) // 64 for x in intents)
    assert prefix_blocks > eng.kv.num_blocks     # the distinct prefixes outgrow the pool

    async def serve():                           # the server path keeps prefixes cached
        return [await planner.plan(x) for x in intents]
    for d in asyncio.run(serve()):
        validate_dag(d, names)
    planner._stop.set()
    eng.drop_prefixes()
    assert eng.alloc.num_free == eng.kv.num_blocks


def test_preemption_by_recompute_under_a_small_kv_pool(monkeypatch):
    """A pool too small for every admitted request's growth: requests are
    preempted (blocks freed, history recomputed later, shared prefix blocks
    kept) and the greedy plans equal a large pool's; a pool that cannot hold
    one request fails it cleanly; no block leaks either way.  (Pool sizes for
    the full model view's token counts.)"""
    import mcp_amd.planner.grammar as grammar
    monkeypatch.setattr(grammar, "COMPACT", False)
    reg = MemoryRegistry(synthetic_registry(5, seed=7))
    intents = [synthetic_intent(i) for i in range(8)]

    def run(nb):
        eng = LLMEngine(LlamaModel.random("tiny", "cpu", seed=1), num_blocks=nb, max_batch=8,
                        temperature=0.0, graphs=False)
        pl = LocalPlanner(eng, reg, max_nodes=4)
        try:
            return pl.plan_many(intents), eng
        except RuntimeError as e:
            return e, eng
    big, eng_big = run(256)
    small, eng = run(14)
    assert eng_big.stats["preemptions"] == 0 and eng.stats["preemptions"] > 0
    assert small == big
    assert eng.alloc.num_free == 14
    err, eng = run(9)
    assert isinstance(err, RuntimeError) and "KV cache exhausted" in str(err)
    assert eng.alloc.num_free == 9 and not eng.running and not eng.waiting


def _distinct_prefix_requests(eng, n):
    """n requests whose registry prefixes differ (own registries), each prefix
    longer than one block with a partial tail."""
    out = []
    for i in range(n):
        reg = MemoryRegistry(synthetic_registry(4 + i, seed=20 + i))
        pl = LocalPlanner(eng, reg, max_nodes=2)
        dec, ptoks, stoks = pl.prepare(synthetic_intent(300 + i))
        assert len(ptoks) > 64 and len(ptoks) % 64
        out.append((dec, ptoks, stoks))
    return out


def test_tail_copies_never_alias_when_evicted_prefixes_materialise_together():
    """two requests whose cached prefixes were evicted before
    they materialise in the same step.  Freeing a tail source right away let
    the LIFO pool hand it to the next request's tail copy, so the step's copy
    list held (t_a -> n_a) and (t_b -> t_a), which run in parallel on the GPU.
    No block may be both a source and a destination in one step, and the
    plans must equal those of an engine that never evicted."""
    import mcp_amd.engine.engine as engmod
    results = []
    for evict in (False, True):
        eng = LLMEngine(LlamaModel.random("tiny", "cpu", seed=1), num_blocks=128, max_batch=8,
                        temperature=0.0, graphs=False)
        reqs = _distinct_prefix_requests(eng, 3)
        seqs = [eng.submit(d, s, prefix_tokens=p) for d, p, s in reqs]
        pairs = []
        real = engmod.ops.copy_blocks

        def spy(kv, src, dst):
            pairs.append((src.tolist(), dst.tolist()))
            return real(kv, src, dst)
        engmod.ops.copy_blocks = spy
        try:
            while any(not e.computed for e in eng.prefixes.values()):
                eng.step()
            if evict:
                eng.drop_prefixes()                # entries gone: requests hold the last refs
            eng.run()
        finally:
            engmod.ops.copy_blocks = real
        assert pairs, "the tail blocks were never copied"
        for src, dst in pairs:
            assert not set(src) & set(dst), (src, dst)
            assert len(set(dst)) == len(dst)
        assert all(q.error is None for q in seqs)
        eng.drop_prefixes()
        assert eng.alloc.num_free == eng.kv.num_blocks
        results.append([q.result for q in seqs])
    assert results[0] == results[1]


def test_evict_prefixes_keeps_entries_that_free_nothing():
    """an entry whose blocks running requests still share
    frees nothing; evicting it would only make later requests recompute it."""
    eng = LLMEngine(LlamaModel.random("tiny", "cpu", seed=1), num_blocks=64, max_batch=8,
                    temperature=0.0, graphs=False)
    (d, p, s), = _distinct_prefix_requests(eng, 1)
    q = eng.submit(d, s, prefix_tokens=p)
    e = eng.prefixes[tuple(p)]
    assert not eng._evict_prefixes(eng.alloc.num_free + 1)   # job + request hold every block
    assert tuple(p) in eng.prefixes
    eng.run()
    assert q.error is None and tuple(p) in eng.prefixes and e.computed
    assert eng._evict_prefixes(eng.alloc.num_free + 1)       # unused now: its blocks come back
    assert tuple(p) not in eng.prefixes and eng.alloc.num_free == eng.kv.num_blocks


def test_pool_pressure_releases_idle_prefix_holders_instead_of_failing(monkeypatch):
    """a request that fits the pool on its own must not fail
    with 'KV cache exhausted' because waiting requests hold references to
    their (distinct) prefixes; those are released and recomputed later.  (The
    full model view's prompt / plan sizes, for which 40 blocks is the pressure
    point.)"""
    import mcp_amd.planner.grammar as grammar
    monkeypatch.setattr(grammar, "COMPACT", False)
    eng = LLMEngine(LlamaModel.random("tiny", "cpu", seed=1), num_blocks=40, max_batch=1,
                    temperature=0.0, graphs=False)
    reqs = _distinct_prefix_requests(eng, 6)
    need = max((len(p) + len(s)) // 64 + 4 for _, p, s in reqs)
    assert sum(len(p) // 64 + 1 for _, p, _ in reqs) + need > eng.kv.num_blocks
    seqs = [eng.submit(d, s, prefix_tokens=p) for d, p, s in reqs]
    eng.run()
    assert all(q.done and q.error is None for q in seqs), [q.error for q in seqs]
    assert eng.stats.get("released", 0) > 0
    eng.drop_prefixes()
    assert eng.alloc.num_free == eng.kv.num_blocks


def test_block_level_prefix_reuse_across_different_prefixes():
    """prompts whose retrieved service lists start alike share
    their leading full KV blocks.  A second prefix that extends the first one's
    services reuses every full block of the first (its prefix job computes
    only the rest, from the shared keys on), and greedy plans equal those of
    an engine that recomputes every prefix (MCP_BLOCK_REUSE=0 semantics)."""
    svc = sorted(synthetic_registry(12, seed=9), key=lambda r: r.name)   # registries list by name
    lists = [svc[:6], svc[:6] + svc[8:11], svc[:4] + svc[6:9]]
    out = []
    for reuse in (False, True):
        eng = LLMEngine(LlamaModel.random("tiny", "cpu", seed=1), num_blocks=256, max_batch=8,
                        temperature=0.0, graphs=False)
        eng.block_reuse = reuse
        seqs = []
        for i, cands in enumerate(lists):
            reg = MemoryRegistry(cands)
            pl = LocalPlanner(eng, reg, max_nodes=3)
            dec, ptoks, stoks = pl.prepare(synthetic_intent(40 + i))
            seqs.append(eng.submit(dec, stoks, prefix_tokens=ptoks))
            eng.run()                         # each prefix computed before the next arrives
        assert all(q.error is None for q in seqs)
        out.append([q.result for q in seqs])
        if reuse:
            e0, e1, e2 = (eng.prefixes[k] for k in list(eng.prefixes)[:3])
            assert e1.shared == e0.length // 64 and e1.blocks[:e1.shared] == e0.blocks[:e1.shared]
            assert 0 < e2.shared < e0.length // 64
            assert eng.stats["prefix_blocks_reused"] == e1.shared + e2.shared
        else:
            assert eng.stats.get("prefix_blocks_reused", 0) == 0
        eng.drop_prefixes()
        assert eng.alloc.num_free == eng.kv.num_blocks
    assert out[0] == out[1]


def test_chunked_prefill_caps_prompt_tokens_beside_decoding_requests(monkeypatch):
    """with MCP_PREFILL_CHUNK, requests still in their
    prompt take at most that many prompt tokens per step while other requests
    are decoding; the plans are the same greedy plans as unchunked."""
    reg = MemoryRegistry(synthetic_registry(12, seed=5))
    first = [synthetic_intent(i) for i in range(3)]
    late = [synthetic_intent(100 + i) for i in range(3)]
    out, steps, worst = [], [], []
    for chunk in ("0", "24"):
        monkeypatch.setenv("MCP_PREFILL_CHUNK", chunk)
        torch.manual_seed(0)
        model = LlamaModel.random("tiny", "cpu", seed=1)
        eng = LLMEngine(model, num_blocks=256, max_batch=16, temperature=0.0, graphs=False)
        assert eng.prefill_chunk == int(chunk)
        planner = LocalPlanner(eng, reg, max_nodes=3)
        seqs = planner.submit_many(first)
        while not all(q.n_samples > 0 for q in seqs):
            eng.step()
        seen = []
        real = eng._schedule_launch_inner

        def rec(cohort, real=real, seen=seen):
            before = {id(q): (q.n_samples, len(q.pending)) for q in eng.running}
            L = real(cohort)
            if L is not None:
                decoding = any(q.n_samples > 0 for q in eng.running)
                pre = sum(t for q, t in L.batch_seqs
                          if q.decoder is not None and before.get(id(q), (1, 0))[0] == 0)
                seen.append((decoding, pre))
            return L
        eng._schedule_launch_inner = rec
        seqs += planner.submit_many(late)
        eng.run()
        assert all(q.done and q.error is None for q in seqs)
        out.append([q.result for q in seqs])
        steps.append(eng.stats["steps"])
        worst.append(max((pre for dec, pre in seen if dec), default=0))
    assert out[0] == out[1]
    assert worst[0] > 24 >= worst[1], worst
    assert steps[1] > steps[0]


def test_decode_priority_prefill_budget_shrinks_with_decoders(monkeypatch):
    """MCP_PREFILL_DECODE_REF makes the per-step prompt
    budget shrink as decoding requests grow (chunk while <= ref decode, chunk
    * ref / n beyond, floored at MCP_PREFILL_MIN); plans stay the greedy plans."""
    monkeypatch.setenv("MCP_PREFILL_CHUNK", "512")
    monkeypatch.setenv("MCP_PREFILL_DECODE_REF", "4")
    monkeypatch.setenv("MCP_PREFILL_MIN", "64")
    model = LlamaModel.random("tiny", "cpu", seed=1)
    eng = LLMEngine(model, num_blocks=256, max_batch=16, temperature=0.0, graphs=False)
    assert [eng.prefill_budget(n) for n in (1, 4, 8, 16, 32, 64)] == [512, 512, 256, 128, 64, 64]
    monkeypatch.setenv("MCP_PREFILL_DECODE_REF", "0")
    eng0 = LLMEngine(model, num_blocks=256, max_batch=16, temperature=0.0, graphs=False)
    assert eng0.prefill_budget(64) == 512
    reg = MemoryRegistry(synthetic_registry(12, seed=5))
    intents = [synthetic_intent(i) for i in range(6)]
    outs = []
    for ref in ("0", "1"):
        monkeypatch.setenv("MCP_PREFILL_CHUNK", "16")
        monkeypatch.setenv("MCP_PREFILL_DECODE_REF", ref)
        monkeypatch.setenv("MCP_PREFILL_MIN", "8")
        torch.manual_seed(0)
        e = LLMEngine(LlamaModel.random("tiny", "cpu", seed=1), num_blocks=256, max_batch=16,
                      temperature=0.0, graphs=False)
        planner = LocalPlanner(e, reg, max_nodes=3)
        seqs = planner.submit_many(intents[:3])
        while not all(q.n_samples > 0 for q in seqs):
            e.step()
        seqs += planner.submit_many(intents[3:])
        e.run()
        assert all(q.done and q.error is None for q in seqs)
        outs.append([q.result for q in seqs])
    assert outs[0] == outs[1]


def test_prep_thread_gives_the_same_plans(monkeypatch):
    """MCP_PREP_THREAD=1: retrieval, grammar and tokenisation run on a prep
    thread beside the engine thread; concurrent async plans are the greedy
    plans of the in-line path."""
    from mcp_amd.retrieval.store import SchemaIndex
    reg = MemoryRegistry(synthetic_registry(60, seed=7))
    intents = [synthetic_intent(300 + i) for i in range(8)]
    outs = []
    for on in ("0", "1"):
        monkeypatch.setenv("MCP_PREP_THREAD", on)
        model = LlamaModel.random("tiny", "cpu", seed=1)
        eng = LLMEngine(model, num_blocks=256, max_batch=8, temperature=0.0, graphs=False)
        retr = SchemaIndex(reg, dim=64, device="cpu")
        retr.refresh()
        planner = LocalPlanner(eng, reg, max_nodes=3, retriever=retr, retrieval_threshold=8, topk=6)
        assert planner.prep_thread == (on == "1")

        async def serve():
            return await asyncio.gather(*[planner.plan(x) for x in intents])
        outs.append(asyncio.run(serve()))
        asyncio.run(planner.aclose())
    assert outs[0] == outs[1]


def test_lookahead_outcome_mismatch_fails_only_that_request(monkeypatch):
    """a sampled token that is no outcome of the pending choice
    (impossible under the grammar's allowed sets; forced here) fails only that
    request with a clear error, the engine leaves lookahead and finishes the
    others, and every KV block comes back."""
    from mcp_amd.engine import native
    if not native.available():
        pytest.skip("native runtime not built")
    reg = MemoryRegistry(synthetic_registry(7, seed=4))
    model = LlamaModel.random("tiny", "cpu", seed=1)
    eng = LLMEngine(model, num_blocks=256, max_batch=16, temperature=0.0, lookahead=True)
    planner = LocalPlanner(eng, reg, max_nodes=4, min_nodes=2)
    real = eng._wait_tokens
    state = {"done": False}

    def corrupt(L):
        toks = real(L)
        import inspect
        if not state["done"] and inspect.stack()[1].function == "_step_look" and toks:
            state["done"] = True
            toks = list(toks)
            toks[0] = -12345                          # no outcome carries this token
        return toks
    monkeypatch.setattr(eng, "_wait_tokens", corrupt)
    seqs = planner.submit_many([synthetic_intent(i) for i in range(3)])
    eng.run()
    assert state["done"], "lookahead never ran"
    errs = [q for q in seqs if q.error]
    assert len(errs) == 1 and "not an outcome" in errs[0].error
    assert "device error word" in errs[0].error and "lookahead_device_errors" in eng.stats
    assert all(q.done for q in seqs) and sum(q.result is not None for q in seqs) == 2
    assert not eng._look and not eng.inflight
    eng.drop_prefixes()
    assert eng.alloc.num_free == eng.kv.num_blocks
