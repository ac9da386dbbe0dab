"""Host time of the engine's own hipGraph replays (config 2 shape): which part
of the captured decode step keeps ``CUDAGraph.replay()`` on the host for the
whole forward (r5g1: 3.6 ms per replay in engine.launch, against ~80 us for a
graph of 192 of the same GEMM kernels, tools/probes/probe_graph_launch.py).

For the buckets the single-intent run used: the replay as captured, and
re-captures of the same step's pieces (forward only, the sampler only, the
forward without attention) on the bucket's static buffers.
"""
import json
import time

import torch

from mcp_amd import ops
from mcp_amd.engine.engine import LLMEngine
from mcp_amd.models.llama import LlamaModel
from mcp_amd.planner.local import LocalPlanner
from mcp_amd.registry.registry import MemoryRegistry
from bench_serve import synthetic_intent, synthetic_registry


def timed(g, reps=7):
    rows = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        rows.append((t1 - t0, time.perf_counter() - t0))
    rows.sort(key=lambda r: r[1])
    h, tot = rows[len(rows) // 2]
    return round(h * 1e6, 1), round(tot * 1e6, 1)


def capture(fn, pool=None):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, pool=pool):
        fn()
    return g


def main():
    dev = torch.device("cuda", 0)
    model = LlamaModel.random("llama3-8b", dev, seed=0)
    engine = LLMEngine(model, max_batch=512, max_step_tokens=16384, temperature=0.2, seed=0)
    reg = MemoryRegistry(synthetic_registry(10, seed=1))
    planner = LocalPlanner(engine, reg, max_nodes=5, min_nodes=5)
    engine.warm_graphs(contexts=(2048,))
    gr = engine.graphs
    r0 = gr.replays
    planner.plan_many([synthetic_intent(-1)])
    planner.plan_many([synthetic_intent(-2)])
    print(json.dumps({"replays_in_two_plans": gr.replays - r0, "buckets": len(gr._b)}), flush=True)
    used = [k for k, e in gr._b.items() if k[0] <= 32]
    for key in used[:6]:
        e = gr._b[key]
        h, tot = timed(e.graph)
        row = {"key": list(key), "as_captured_host_us": h, "as_captured_total_us": tot}
        hid = {}

        def fwd():
            hid["h"] = model.forward(e.dstep, engine.kv)
        g = capture(fwd)
        row["forward_only"] = timed(g)

        def smp():
            ops.sample_allowed(hid["h"], model.w.lm_head, e.dstep.allow_ptr, e.dstep.allow_ids,
                               e.dstep.sample_ctr, 0.2, 0)
        if hid["h"] is not None:
            g = capture(smp)
            row["sample_only"] = timed(g)

        def cow():
            ops.copy_blocks(engine.kv.data, e.csrc, e.cdst)
        g = capture(cow)
        row["copy_blocks_only"] = timed(g)

        st = e.dstep
        T = st.token_ids.numel()
        D = model.cfg.head_dim
        xx = torch.randn(T, model.cfg.hidden, device=dev, dtype=torch.bfloat16)
        q = torch.empty(T, model.hq, D, device=dev, dtype=torch.bfloat16)
        ssx = torch.zeros(T, dtype=torch.int64, device=dev)
        kc, vc = engine.kv.layer(0)
        lw = model.w.layers[0]

        def qkv32():
            for _ in range(32):
                ops.qkv_rope(xx, lw.wqkv, st.positions, st.slots, model.cos_sin, q, kc, vc,
                             model.hq, model.hkv, D, ss_in=ssx, eps=1e-5)
        row["qkv_rope_x32"] = timed(capture(qkv32))

        def attn32():
            for _ in range(32):
                ops.paged_attention(q, kc, vc, st.attn, model.scale)
        row["attention_x32"] = timed(capture(attn32))

        def emb():
            ops.embedding(st.token_ids, model.w.embed)
            ops.row_sumsq(xx, ssx)
            torch.zeros(33, 2, T, dtype=torch.int64, device=dev)
        row["embed_sumsq_zeros"] = timed(capture(emb))
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
