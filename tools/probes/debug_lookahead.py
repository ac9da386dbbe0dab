"""Lookahead engine on the GPU, eager steps: check every sampler call's inputs
(finite hidden rows, monotone allowed pointers) and print the step views of
the first bad one."""
import itertools
import sys

import torch

from mcp_amd import ops
from mcp_amd.engine import engine as engine_mod
from mcp_amd.engine.engine import LLMEngine
from mcp_amd.models.llama import LlamaModel
from mcp_amd.planner.local import LocalPlanner
from mcp_amd.planner.prompt import synthetic_intent
from mcp_amd.registry import MemoryRegistry, synthetic_registry

orig_sample = ops.sample_allowed
orig_select = ops.branch_select
last = {}


def select(prev_tok, tab, n, dstep, err):
    orig_select(prev_tok, tab, n, dstep, err)
    torch.cuda.synchronize()
    last["tab"] = tab.tolist()
    last["prev"] = prev_tok.tolist()[:16]
    last["views"] = {k: v.tolist()[:40] for k, v in (
        ("ids", dstep.token_ids), ("ql", dstep.attn.q_len), ("cl", dstep.attn.ctx_len),
        ("rows", dstep.logit_rows), ("aptr", dstep.allow_ptr), ("aids", dstep.allow_ids),
        ("pos", dstep.positions), ("slots", dstep.slots), ("qs", dstep.attn.q_start))}
    last["splits"] = dstep.attn.kv_splits
    last["own"] = dstep.attn.own_tiles
    last["work"] = [(nw, ws.tolist(), wq.tolist()) for nw, ws, wq in dstep.attn.work_lists()]


def sample(hidden, W, ap, ai, ctr, t, seed, **kw):
    torch.cuda.synchronize()
    fin = torch.isfinite(hidden.float()).all(dim=1).tolist()
    a = ap.tolist()
    r = orig_sample(hidden, W, ap, ai, ctr, t, seed, **kw)
    torch.cuda.synchronize()
    if not all(fin) or any(x < 0 for x in r.tolist()):
        print("BAD sample: finite rows", fin, "aptr", a[:12], "tokens", r.tolist(), flush=True)
        print("last select:", last, flush=True)
        sys.exit(3)
    return r


ops.sample_allowed = sample
ops.branch_select = select
graphs = "--graphs" in sys.argv
model = LlamaModel.random("tiny", "cuda", seed=3)
reg = MemoryRegistry(synthetic_registry(8, seed=2))
engine_mod._uid = itertools.count(1)
eng = LLMEngine(model, num_blocks=512, max_batch=32, temperature=0.0, graphs=graphs,
                pipeline=False, lookahead=True)
planner = LocalPlanner(eng, reg, max_nodes=4, min_nodes=2)
for i in range(2):
    print(planner.plan_many([synthetic_intent(i)])[0], flush=True)
print("stats", eng.stats, flush=True)
