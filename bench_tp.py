#!/usr/bin/env python3
"""BASELINE config 4: Llama-3-70B planner at TP=8 over xGMI, 50-service
registry, execution with retries + ordered fallbacks.

    python bench_tp.py --gpus 8 --model llama3-70b

(``--gpus N`` starts the N ranks itself, parallel.launch; torchrun works too.)

One process per GPU.  Rank 0 is the TP driver (scheduler, grammar, sampling);
ranks 1..7 mirror the sharded forward from broadcast step descriptors
(engine.tp).  The row-parallel projections all-reduce over RCCL.  After
planning, rank 0 executes every DAG through the orchestrator against mock
services with injected faults (5xx on the first attempt of some services,
dead primaries with working fallbacks) so per-node retries and ordered
fallbacks run.  Without torchrun it runs TP=1 on one GPU (70B bf16 fits in
288 GB).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import zlib
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import mcp_amd  # noqa: E402,F401


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--services", type=int, default=50)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--max-nodes", type=int, default=6)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--seq-parallel", action="store_true",
                    help="Megatron sequence parallelism (reduce-scatter / all-gather) for TP > 1")
    ap.add_argument("--gpus", type=int, default=1, help="TP degree = ranks (one per GPU); N > 1 self-launches")
    args = ap.parse_args()
    from mcp_amd.parallel.launch import check_devices, self_launch
    rc = self_launch(args.gpus)
    if rc is not None:
        sys.exit(rc)
    check_devices(int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1"))),
                  int(os.environ.get("LOCAL_RANK", "0")))

    from mcp_amd.engine.engine import LLMEngine
    from mcp_amd.engine.kv_cache import KVCache
    from mcp_amd.engine.tp import agree_num_blocks, worker_loop
    from mcp_amd.models.llama import LlamaModel, get_config
    from mcp_amd.parallel.comm import StepBroadcaster, init_distributed

    rank, world, local_rank, dev = init_distributed()

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
    tp = world
    group = dist.group.WORLD if world > 1 else None
    t0 = time.time()
    if args.seq_parallel:
        os.environ["MCP_SEQ_PARALLEL"] = "1"
    model = LlamaModel.random(args.model, dev, seed=args.seed, tp_rank=rank, tp=tp, tp_group=group)
    sync()
    log(f"[rank {rank}] {args.model} TP={tp} shard ready in {time.time() - t0:.1f}s")
    cfg = get_config(args.model)
    per_block = KVCache.bytes_per_block(cfg.layers, model.hkv, cfg.head_dim)
    nb = agree_num_blocks(per_block, dev, group, cap=65536)
    bcast = StepBroadcaster(group, dev) if world > 1 else None
    if rank != 0:
        kv = KVCache(cfg.layers, model.hkv, cfg.head_dim, nb, dev)
        n = worker_loop(model, kv, bcast)
        log(f"[rank {rank}] worker done after {n} steps")
        dist.destroy_process_group()
        return

    import httpx
    from mcp_amd.orchestrator import Orchestrator, validate_dag
    from mcp_amd.planner.local import LocalPlanner
    from mcp_amd.planner.prompt import synthetic_intent
    from mcp_amd.registry import MemoryRegistry, synthetic_registry

    eng = LLMEngine(model, num_blocks=nb, max_batch=args.batch + 8, max_step_tokens=16384,
                    temperature=0.2, seed=args.seed, bcast=bcast)
    reg = MemoryRegistry(synthetic_registry(args.services, seed=4))
    planner = LocalPlanner(eng, reg, max_nodes=args.max_nodes, retrieval_threshold=10 ** 9)
    names = [s.name for s in reg.list_services()]
    t0 = time.perf_counter()
    ncap = eng.warm_graphs(contexts=(8192,))         # server start-up capture (planner.local)
    log(f"[rank 0] start-up graph capture: {ncap} graphs in {time.perf_counter() - t0:.1f}s")
    def one_step(base):
        """One closed batch: submit every intent, run the engine (and, through
        the step broadcasts, every worker rank) dry."""
        seqs = planner.submit_many([synthetic_intent(base + i) for i in range(args.batch)])
        eng.run()
        return seqs

    for w in range(args.warmup):
        one_step(10_000 + w * args.batch)
    sync()
    t = time.perf_counter()
    seqs_all = []
    for s in range(args.steps):
        ts = time.perf_counter()
        seqs_all += one_step(s * args.batch)
        log(f"[rank 0] step {s}: {(time.perf_counter() - ts) * 1e3:.0f} ms")
    sync()
    elapsed = time.perf_counter() - t
    eng.shutdown_workers()
    for q in seqs_all:
        if q.error:
            raise RuntimeError(q.error)
        validate_dag(q.result, names)
    dags = [q.result for q in seqs_all]
    # each timed request's own intent -> DAG latency (submit -> DAG parsed), as
    # in bench.py; rank 0 is the only driver, so its requests are all of them
    lats = [q.t_done - q.t_submit for q in seqs_all]

    # ---- execute every plan with injected faults: retries + ordered fallbacks
    attempts = {}

    def handler(request: httpx.Request):
        host = request.url.host
        attempts[host] = attempts.get(host, 0) + 1
        h = zlib.crc32(host.encode()) % 7                    # stable across runs (str hash is salted)
        if h == 0 and not host.endswith("fallback"):          # dead primary
            return httpx.Response(503)
        if h == 1 and attempts[host] % 2 == 1:                # flaky: fails every other call
            return httpx.Response(500)
        return httpx.Response(200, json={"svc": host})

    async def run_all():
        orch = Orchestrator(client=httpx.AsyncClient(transport=httpx.MockTransport(handler)),
                            retries=1, concurrent_generations=True, registry=reg,
                            use_registry_fallback=True)
        out = {"ok": 0, "with_errors": 0, "aborted": 0}
        for d in dags:
            try:
                r = await orch.execute(d, {"user_id": "u1", "order_id": "o1", "amount": 10})
                out["with_errors" if r["errors"] else "ok"] += 1
            except Exception:
                out["aborted"] += 1
        await orch.aclose()
        return out
    logging_level = os.environ.get("MCP_BENCH_LOG", "WARNING")
    import logging
    logging.getLogger("httpx").setLevel(logging_level)
    logging.getLogger("orchestrator").setLevel(logging_level)
    exec_stats = asyncio.run(run_all())
    print(json.dumps({
        "config": "llama3-70b TP planner, 50-service registry, retries + ordered fallbacks",
        "model": args.model, "tp": tp, "seq_parallel": model.seq_parallel, "services": args.services, "batch": args.batch,
        "plans_per_s": round(len(dags) / elapsed, 3),
        "p50_latency_ms": round(statistics.median(lats) * 1e3, 1) if lats else None,
        "p99_latency_ms": round(statistics.quantiles(lats, n=100)[98] * 1e3, 1)
        if len(lats) >= 2 else None,
        "tokens": eng.stats["tokens"], "execution": exec_stats,
    }), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
