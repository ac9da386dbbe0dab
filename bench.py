#!/usr/bin/env python3
"""Headline benchmark: plans/sec (whole node) + p50 intent->DAG latency,
Llama-3-8B planner at TP=1 (BASELINE.json ``metric``; configs 2 and 5).

One *step* = one batch of ``--batch`` synthetic intents per GPU planned end to
end on that GPU's replica (data parallel: one process and one TP=1
Llama-3-8B per GPU).  ``--gpus N`` with N > 1 starts the N ranks itself
(parallel.launch: fresh child processes, one per GPU, before anything touches
HIP); under torchrun the ranks come from the launcher instead.  By default the batches
run strictly one after another; ``--overlap F`` admits batch k+1 once at most
a fraction F of batch k is still decoding (continuous batching, the serving
engine's normal mode): the GPU no longer idles through a batch's tail of short
decode steps (+3 % plans/s at F = 0.4) at the cost of p50 latency (+8 %),
measured in profiles/bench_overlap_sweep.jsonl.  Per request:

    intent -> prompt (10-service registry) -> tokenize -> prefix + suffix prefill
    -> grammar-constrained decode with jump-forward (temperature 0.2)
    -> valid T2 DAG JSON (checked after timing)

Everything a request needs happens inside the timed step, including the
prefill of the shared registry prompt (the prefix cache is dropped after each
batch).  Weights are random-init bf16 of the exact Llama-3-8B architecture
(no checkpoints offline); intents are synthetic.  The value reported is the
whole-job aggregate: sum over ranks of plans / max-over-ranks timed span; the
p50 is the median over ALL ranks' timed requests of each request's own
submit -> DAG time (``t_done - t_submit``).  ``--device cpu`` runs the same
code on CPU ranks over gloo (the launcher's CPU test).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

METRIC = "plans/sec (whole node) + p50 intent->DAG latency, Llama-3-8B planner TP=1"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _pin_cpus(local_rank: int, local_world: int):
    """One rank per GPU: give each rank its own contiguous slice of the CPUs this
    process may use, so the ranks' host paths (scheduler, grammar, kernel
    launches) do not migrate onto each other's cores.  MCP_PIN_CPUS=0 disables."""
    if os.environ.get("MCP_PIN_CPUS", "1") == "0" or not hasattr(os, "sched_setaffinity"):
        return
    cpus = sorted(os.sched_getaffinity(0))
    n = len(cpus) // max(1, local_world)
    if n >= 2:
        os.sched_setaffinity(0, cpus[local_rank * n:(local_rank + 1) * n])


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU) on this node; N > 1 self-launches N processes "
                         "unless already started by torchrun")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=256, help="concurrent intents per GPU per step")
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: the same code path on CPU ranks over gloo (launcher tests)")
    ap.add_argument("--services", type=int, default=10)
    ap.add_argument("--min-nodes", type=int, default=5,
                    help="plans have between min and max nodes; min == max fixes the DAG size so "
                         "the work per plan does not depend on the random weights' choices")
    ap.add_argument("--max-nodes", type=int, default=5)
    ap.add_argument("--max-step-tokens", type=int, default=4096,
                    help="token budget per engine step; 4096 = 16 M-tiles of 256 -> whole waves on 256 CUs")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--overlap", type=float, default=0.0,
                    help="submit the next batch once this fraction of the current one is still "
                         "running (0: closed batches)")
    return ap.parse_args(argv)


def main():
    args = parse_args()
    from mcp_amd.parallel.launch import check_devices, self_launch
    rc = self_launch(args.gpus)          # parent of N ranks: never touches the GPU
    if rc is not None:
        sys.exit(rc)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world != args.gpus:
        log(f"[rank {rank}] --gpus {args.gpus} but the launcher started {world} ranks: using {world}")
    cuda = args.device == "cuda"
    if cuda:
        check_devices(local_world, local_rank)
    if world > 1:
        _pin_cpus(local_rank, local_world)
        if cuda:
            torch.cuda.set_device(local_rank)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local_rank) if cuda else torch.device("cpu")

    def sync():
        if cuda:
            torch.cuda.synchronize()

    from mcp_amd.engine.engine import LLMEngine
    from mcp_amd.models.llama import LlamaModel, get_config
    from mcp_amd.orchestrator import validate_dag
    from mcp_amd.planner.local import LocalPlanner
    from mcp_amd.planner.prompt import synthetic_intent
    from mcp_amd.registry import MemoryRegistry, synthetic_registry
    from mcp_amd.utils.heap import settle as settle_heap
    from mcp_amd.planner.grammar import COMPACT as grammar_compact

    t0 = time.time()
    model = LlamaModel.random(args.model, dev, seed=args.seed)
    sync()
    log(f"[rank {rank}] {args.model} random-init on {dev} in {time.time() - t0:.1f}s "
        f"({model.cfg.params() / 1e9:.2f}B params)")
    kw = {} if cuda else {"num_blocks": 64 + 8 * args.batch}
    engine = LLMEngine(model, max_batch=2 * args.batch + 8, max_step_tokens=args.max_step_tokens,
                       temperature=0.2, seed=args.seed + rank, **kw)
    log(f"[rank {rank}] KV cache: {engine.kv.num_blocks} blocks x 64 tokens "
        f"({engine.kv.data.numel() * 2 / 1e9:.1f} GB)")
    reg = MemoryRegistry(synthetic_registry(args.services, seed=1))
    planner = LocalPlanner(engine, reg, max_nodes=args.max_nodes, min_nodes=args.min_nodes)
    names = [s.name for s in reg.list_services()]

    def one_step(step_idx):
        """One closed batch: submit every intent, run the engine dry."""
        base = (step_idx * world + rank) * args.batch
        intents = [synthetic_intent(base + i) for i in range(args.batch)]
        tok0 = engine.stats["tokens"]
        t = time.perf_counter()
        # the batch prefix job runs on the GPU while the suffixes tokenise (MCP_LAUNCH_AHEAD=0: off)
        seqs = planner.submit_many(intents, launch_ahead=os.environ.get("MCP_LAUNCH_AHEAD", "1") == "1")
        engine.run()
        return seqs, time.perf_counter() - t, engine.stats["tokens"] - tok0

    # server start-up (planner.local / bench_serve): capture the hipGraph
    # buckets before any request, so no timed step pays for a lazy capture
    t0 = time.time()
    ncap = engine.warm_graphs(contexts=(2048,)) if cuda else 0
    log(f"[rank {rank}] start-up graph capture: {ncap} graphs in {time.time() - t0:.1f}s")
    for w in range(args.warmup):
        _, dt, toks = one_step(-1 - w)
        log(f"[rank {rank}] warmup {w}: {dt * 1e3:.0f} ms, {toks} tokens")
    settle_heap()                  # as a server does once it is up (utils/heap.py)
    cap0 = engine.stats.get("graph_captures", 0)
    seqs_all = []
    if world > 1:
        dist.barrier()
    sync()
    t_start = time.perf_counter()
    tok0, steps0 = engine.stats["tokens"], engine.stats["steps"]
    if args.overlap <= 0:
        for s in range(args.steps):
            seqs, dt, toks = one_step(s)
            seqs_all += seqs
            log(f"[rank {rank}] step {s}: {dt * 1e3:.0f} ms, {toks} tokens")
    else:
        # continuous batching: drive the engine here; admit batch k+1 once at
        # most `overlap` of batch k is still running
        batches, t_sub = [], []
        nxt = 0

        def submit_next():
            nonlocal nxt
            base = (nxt * world + rank) * args.batch
            batches.append(planner.submit_many([synthetic_intent(base + i) for i in range(args.batch)]))
            t_sub.append(time.perf_counter())
            nxt += 1

        submit_next()
        while True:
            if nxt < args.steps:
                live = sum(1 for q in batches[-1] if not q.done)
                if live <= args.overlap * args.batch:
                    submit_next()
            if not engine.has_work():
                if nxt >= args.steps:
                    break
                continue
            if engine.step() == 0 and not engine.waiting and not engine.inflight:
                if any(not q.pending for q in engine.running):
                    raise RuntimeError("engine stalled with sequences that have no pending tokens")
        for k, b in enumerate(batches):
            seqs_all += b
            log(f"[rank {rank}] batch {k}: done {max(q.t_done for q in b) - t_sub[k]:.3f} s after submit")
    tokens = engine.stats["tokens"] - tok0
    log(f"[rank {rank}] {engine.stats['steps'] - steps0} engine steps, {tokens} tokens, "
        f"{engine.stats.get('graph_captures', 0) - cap0} lazy graph captures in the timed steps")
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    st = engine.stats
    log(f"[rank {rank}] engine totals: " + ", ".join(f"{k}={v:.3f}" if isinstance(v, float) else f"{k}={v}"
                                                  for k, v in st.items()))
    # correctness after timing: every plan is a valid T2 DAG over the registry
    for q in seqs_all:
        if q.error:
            raise RuntimeError(q.error)
        validate_dag(q.result, names)
    # each timed request's own intent -> DAG latency (not a bounded metrics window)
    lats = [q.t_done - q.t_submit for q in seqs_all]
    mine = {"elapsed": elapsed, "plans": len(seqs_all), "tokens": tokens, "lats": lats}
    if world > 1:
        every = [None] * world
        dist.all_gather_object(every, mine)
    else:
        every = [mine]
    elapsed_max = max(e["elapsed"] for e in every)
    plans_total = sum(e["plans"] for e in every)
    tokens_total = sum(e["tokens"] for e in every)
    all_lats = [x for e in every for x in e["lats"]]
    p50 = statistics.median(all_lats) if all_lats else float("nan")
    ms_per_step = elapsed_max / args.steps * 1e3
    value = plans_total / elapsed_max
    # workload-invariant throughput: the decoder layers' projection FLOPs per
    # token (qkv, o, gate|up, down; no attention, embedding or LM head) at the
    # measured token rate - moves with engine speed, not with the plan view
    mc = get_config(args.model)
    layer_params = mc.layers * (mc.hidden * (mc.heads + 2 * mc.kv_heads) * mc.head_dim
                                + mc.heads * mc.head_dim * mc.hidden
                                + 3 * mc.hidden * mc.ffn)
    if rank == 0:
        print(json.dumps({
            "metric": METRIC, "value": round(value, 3), "unit": "plans/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic intents, random-init weights",
            "p50_latency_ms": round(p50 * 1e3, 2),
            "p99_latency_ms": round(statistics.quantiles(all_lats, n=100)[98] * 1e3, 2)
            if len(all_lats) >= 2 else None,
            "tokens_per_s": round(tokens_total / elapsed_max, 1),
            "projection_pflops": round(2 * layer_params * tokens_total / elapsed_max / 1e15, 4),
            "batching": "continuous" if args.overlap > 0 else "closed",
            "device": args.device,
            "config": {"model": args.model, "global_batch": args.batch * world,
                       "seq_len": None, "parallelism": f"dp{world}", "tp": 1,
                       "services": args.services, "nodes_per_plan": [args.min_nodes, args.max_nodes],
                       "tokens_per_plan": round(tokens_total / max(1, plans_total), 1),
                       # compact: URLs filled from the registry, not run through
                       # the model (planner/grammar.py; MCP_PLAN_COMPACT=0: full)
                       "plan_view": "compact" if grammar_compact else "full",
                       "temperature": 0.2},
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
