"""Decision lookahead on the GPU (engine MCP_LOOKAHEAD): the outcome-select
kernel (csrc/sampling.hip branch_select_kernel) against its host version, and
the lookahead engine's plans against the synchronous engine's (greedy and
sampled, eager and hipGraph steps)."""
import itertools

import pytest
import torch

from mcp_amd import ops
from mcp_amd.engine import engine as engine_mod
from mcp_amd.engine.batch import AttnMeta, DeviceStep
from mcp_amd.engine.engine import LLMEngine
from mcp_amd.models.llama import LlamaModel
from mcp_amd.orchestrator import validate_dag
from mcp_amd.planner.local import LocalPlanner
from mcp_amd.planner.prompt import synthetic_intent
from mcp_amd.registry import MemoryRegistry, synthetic_registry

pytestmark = pytest.mark.gpu


def _table(rng, n, T_cap):
    """A random outcome table in engine._launch_branch's layout."""
    per, qs = [], 0
    for i in range(n):
        L = int(rng.integers(1, 9))
        nb = int(rng.integers(2, 6))
        toks = rng.choice(1000, size=nb, replace=False).tolist()
        brs = []
        for t in toks:
            ql = int(rng.integers(1, L + 1))
            ids = [t] + rng.integers(0, 1000, size=ql - 1).tolist()
            nxt = rng.integers(0, 1000, size=int(rng.integers(2, 7))).tolist()
            brs.append((t, ids, nxt))
        per.append((i, qs, int(rng.integers(0, 500)), L, brs))
        qs += L
    assert qs <= T_cap
    off = 2 + 6 * n
    tab = [n, 0] + [0] * (6 * n)
    recs, pool = [], []
    base = off + sum(len(p[4]) * (4 + p[3]) for p in per)
    for i, (prow, q0, start, L, brs) in enumerate(per):
        tab[2 + 6 * i: 8 + 6 * i] = [prow, q0, start, L, len(brs), off + len(recs)]
        for t, ids, nxt in brs:
            recs += [t, len(ids), base + len(pool), len(nxt)] + ids + [0] * (L - len(ids))
            pool += nxt
    tab += recs + pool
    return tab, per


def _with_tail(tab, tail_sets):
    """Append the tail section: allowed sets of rows after the lookahead rows."""
    tab = list(tab)
    tab[1] = len(tab)
    rel = [0]
    for a in tail_sets:
        rel.append(rel[-1] + len(a))
    tab += [len(tail_sets)] + rel + [x for a in tail_sets for x in a]
    return tab


def _step(dev, T, S, A):
    z = lambda k: torch.arange(k, dtype=torch.int32, device=dev)  # noqa: E731
    meta = AttnMeta(q_start=z(S), q_len=z(S), ctx_len=z(S), block_table=z(S).view(S, 1), work=[])
    return DeviceStep(token_ids=z(T), positions=z(T), slots=z(T), logit_rows=z(S), attn=meta,
                      allow_ptr=z(S + 1), allow_ids=z(A), sample_ctr=z(S))


@pytest.mark.parametrize("n,tail", [(1, 0), (3, 0), (8, 0), (2, 3)])
def test_branch_select_kernel_matches_host(n, tail):
    import numpy as np
    rng = np.random.default_rng(n)
    tab, per = _table(rng, n, 128)
    tail_sets = [rng.integers(0, 1000, size=int(rng.integers(1, 5))).tolist() for _ in range(tail)]
    if tail:
        tab = _with_tail(tab, tail_sets)
    prev = torch.tensor([p[4][int(rng.integers(0, len(p[4])))][0] for p in per], dtype=torch.int32)
    outs = []
    for dev in ("cpu", "cuda"):
        st = _step(dev, 128, 12, 64)
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        ops.branch_select(prev.to(dev), torch.tensor(tab, dtype=torch.int32, device=dev), n, st, err)
        torch.cuda.synchronize()
        outs.append([x.cpu() for x in (st.token_ids, st.attn.q_len, st.attn.ctx_len, st.logit_rows,
                                       st.allow_ptr, st.allow_ids, st.slots, err)])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert int(outs[1][-1][0]) == 0
    # the selected outcome per sequence
    for i, (_, q0, start, L, brs) in enumerate(per):
        t, ids, nxt = next(b for b in brs if b[0] == int(prev[i]))
        assert outs[1][1][i] == len(ids) and outs[1][2][i] == start + len(ids)
        assert outs[1][3][i] == q0 + len(ids) - 1
        assert outs[1][0][q0:q0 + len(ids)].tolist() == ids
        # rows past the outcome's span: no KV slot
        assert outs[1][6][q0 + len(ids):q0 + L].tolist() == [-1] * (L - len(ids))
        a0, a1 = int(outs[1][4][i]), int(outs[1][4][i + 1])
        assert outs[1][5][a0:a1].tolist() == nxt
    for j, a in enumerate(tail_sets):               # tail rows follow the chosen sets
        a0, a1 = int(outs[1][4][n + j]), int(outs[1][4][n + j + 1])
        assert outs[1][5][a0:a1].tolist() == a


@pytest.mark.parametrize("graphs,temperature", [(False, 0.0), (True, 0.0), (True, 0.2)])
def test_lookahead_engine_matches_synchronous(graphs, temperature, monkeypatch):
    model = LlamaModel.random("tiny", "cuda", seed=3)
    reg = MemoryRegistry(synthetic_registry(8, seed=2))
    intents = [synthetic_intent(i) for i in range(4)]
    out, stats = [], []
    for look in (False, True):
        monkeypatch.setattr(engine_mod, "_uid", itertools.count(1))
        eng = LLMEngine(model, num_blocks=512, max_batch=32, temperature=temperature,
                        graphs=graphs, pipeline=False, lookahead=look)
        planner = LocalPlanner(eng, reg, max_nodes=4, min_nodes=2)
        res = [planner.plan_many([it])[0] for it in intents[:2]]
        res += planner.plan_many(intents)
        torch.cuda.synchronize()
        assert eng.alloc.num_free == eng.kv.num_blocks and not eng._look
        out.append(res)
        stats.append(dict(eng.stats))
    assert stats[1]["lookahead_steps"] > 0
    if graphs:
        assert stats[1]["graph_steps"] > 0
    assert out[0] == out[1]
    names = [s.name for s in reg.list_services()]
    for d in out[1]:
        validate_dag(d, names)


@pytest.mark.parametrize("graphs", [False, True])
def test_lookahead_admits_arrivals_matches_synchronous(graphs, monkeypatch):
    """Requests arriving during lookahead join the next lookahead step; the
    plans equal the synchronous engine's under the same arrival schedule."""
    model = LlamaModel.random("tiny", "cuda", seed=3)
    reg = MemoryRegistry(synthetic_registry(8, seed=2))
    out, admitted = [], []
    for look in (False, True):
        monkeypatch.setattr(engine_mod, "_uid", itertools.count(1))
        eng = LLMEngine(model, num_blocks=512, max_batch=32, temperature=0.2, graphs=graphs,
                        pipeline=False, lookahead=look)
        planner = LocalPlanner(eng, reg, max_nodes=4, min_nodes=2)
        planner.plan_many([synthetic_intent(99)])
        seqs = []
        for i in range(4):
            dec, ptoks, stoks = planner.prepare(synthetic_intent(i))
            seqs.append(eng.submit(dec, stoks, prefix_tokens=ptoks))
            for _ in range(3 + i):
                if eng.has_work():
                    eng.step()
        eng.run()
        torch.cuda.synchronize()
        assert all(q.error is None for q in seqs) and not eng._look
        out.append([q.result for q in seqs])
        admitted.append(eng.stats["lookahead_admitted"])
    assert out[0] == out[1]
    assert admitted[1] > 0
