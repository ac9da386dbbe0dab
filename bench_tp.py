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


# xGMI / RCCL assumptions of the TP prediction (--simulate-rank): the cost
# model of the run-time dispatch, parallel/xgmi_model.py (MCP_XGMI_* overrides)


class _SimAllReduce:
    """Stands in for the TP group's all-reduce on a simulated rank: no data
    moves (the rank's partial sums flow on unreduced - the arithmetic per
    rank is unchanged), capturable in hipGraphs like K12.  ``emulate``: each
    call launches a kernel that holds the CUs a K12 call of that size would
    hold for the xGMI model's time (csrc/custom_allreduce.hip
    comm_emulate_kernel), on the caller's stream - so the row-chunked MLP
    block's comm stream (models/llama.py _mlp_block_overlapped) is measured
    overlapping the GEMMs for real, CU contention included."""

    def __init__(self, emulate: bool = False, tp: int = 1, car_max: int = 0):
        self.emulate, self.tp, self.car_max = emulate, tp, car_max
        self.calls = 0

    def __call__(self, t):
        if self.emulate and t.is_cuda:
            from mcp_amd import ops
            from mcp_amd.parallel import xgmi_model as xm
            nbytes = t.numel() * t.element_size()
            # MCP_CAR_BLOCKS caps the blocks as it caps K12's
            ops.lib().comm_emulate(xm.best(nbytes, self.tp, self.car_max)[1], nbytes,
                                   int(os.environ.get("MCP_CAR_BLOCKS", "0")))
            self.calls += 1
        return None

    def check(self):
        return None

    def graph_safe(self, nbytes):
        return True


def _k12_timer(rank, world, port, sizes, q):
    """Two K12 ranks on this GPU: us per all-reduce of each size (eager,
    both ranks calling together; the flag barriers and kernel launches are
    the real ones, the peer reads hit local HBM instead of xGMI)."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        from mcp_amd.parallel.custom_allreduce import CustomAllReduce
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        car = CustomAllReduce(dist.group.WORLD, "cuda:0", max_bytes=max(sizes))
        out = {}
        for nb in sizes:
            x = torch.randn(nb // 2, device="cuda").bfloat16()
            for _ in range(5):
                car(x)
            torch.cuda.synchronize()
            dist.barrier()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(40):
                car(x)
            e1.record()
            torch.cuda.synchronize()
            out[nb] = e0.elapsed_time(e1) / 40 * 1e3
        car.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, out))
    except Exception as e:  # noqa: BLE001 - reported to the parent
        q.put((rank, repr(e)))


def simulate_rank(args):
    """config 4 at TP = ``--simulate-rank`` predicted on ONE
    GPU.  Rank 0 of the TP group runs alone: its real weight shards (qkv / o /
    gate|up / down divided by tp, random init), its KV heads, the driver's
    scheduler, grammar and sampling, hipGraphs as a TP driver captures them -
    with the all-reduces replaced by no-ops, so the timed batches give the
    rank's compute time.  Every all-reduce the steps would issue (2 per layer
    of [T, H] bf16, the last layer on the sampled rows) is then priced: K12
    path and price come from the xGMI cost model the run-time dispatch uses
    (parallel/xgmi_model.py: K12 one-/two-shot vs RCCL); a pessimistic
    variant prices K12 calls at the two-process time on this one GPU where
    that is higher.  No overlap of communication with compute is assumed."""
    import torch.multiprocessing as mp
    from mcp_amd.engine.engine import LLMEngine
    from mcp_amd.engine.kv_cache import KVCache
    from mcp_amd.models.llama import LlamaModel, get_config, random_weights
    from mcp_amd.orchestrator import validate_dag
    from mcp_amd.parallel.launch import free_port
    from mcp_amd.planner.local import LocalPlanner
    from mcp_amd.planner.prompt import synthetic_intent
    from mcp_amd.registry import MemoryRegistry, synthetic_registry

    tp = args.simulate_rank
    cuda = torch.cuda.is_available()
    dev = torch.device("cuda", 0) if cuda else torch.device("cpu")
    sync = torch.cuda.synchronize if cuda else (lambda: None)
    cfg = get_config(args.model)
    H = cfg.hidden
    t0 = time.time()
    from mcp_amd.parallel.comm import K12_MAX_BYTES
    car_max = int(os.environ.get("MCP_CAR_MAX_BYTES", str(K12_MAX_BYTES)))
    sim_ar = _SimAllReduce(emulate=args.emulate_comm and cuda, tp=tp, car_max=car_max)
    model = LlamaModel(cfg, random_weights(cfg, dev, seed=args.seed, tp_rank=0, tp=tp), dev,
                       0, tp, None, allreduce=sim_ar)
    sync()
    log(f"[sim rank 0 of TP={tp}] {args.model} shard ready in {time.time() - t0:.1f}s")
    per_block = KVCache.bytes_per_block(cfg.layers, model.hkv, cfg.head_dim)
    if cuda:
        free, total = torch.cuda.mem_get_info(dev)
        nb = int(min(65536, (free - 0.1 * total) // per_block))
    else:
        nb = 64 + 8 * args.batch
    eng = LLMEngine(model, num_blocks=nb, max_batch=args.batch + 8, max_step_tokens=16384,
                    temperature=0.2, seed=args.seed, graphs=cuda)
    reg = MemoryRegistry(synthetic_registry(args.services, seed=4))
    planner = LocalPlanner(eng, reg, max_nodes=args.max_nodes, min_nodes=args.min_nodes,
                           retrieval_threshold=10 ** 9)
    names = [s.name for s in reg.list_services()]
    ncap = eng.warm_graphs(contexts=(8192,))
    steps = []
    real = eng._schedule_launch

    def rec(cohort):
        L = real(cohort)
        if L is not None:
            steps.append((L.T, len(L.sample_seqs)))
        return L
    eng._schedule_launch = rec

    def one_step(base):
        seqs = planner.submit_many([synthetic_intent(base + i) for i in range(args.batch)])
        eng.run()
        return seqs
    for w in range(args.warmup):
        one_step(10_000 + w * args.batch)
    sync()
    steps.clear()
    t = time.perf_counter()
    seqs_all = []
    for s in range(args.steps):
        seqs_all += one_step(s * args.batch)
    sync()
    compute_s = time.perf_counter() - t
    for q in seqs_all:
        if q.error:
            raise RuntimeError(q.error)
        validate_dag(q.result, names)
    lats = sorted(q.t_done - q.t_submit for q in seqs_all)

    # ---- every all-reduce of the timed steps
    msgs = []
    for T, ns in steps:
        msgs += [T * H * 2] * (2 * (cfg.layers - 1)) + ([ns * H * 2] * 2 if ns else [])
    from mcp_amd.parallel import xgmi_model as xm
    if sim_ar.emulate:
        # the timed steps ran every all-reduce as an emulated K12 call on the
        # GPU: the measured time IS the prediction (overlap as the model ran it)
        plans = len(seqs_all)
        print(json.dumps({
            "config": "llama3-70b TP planner, 50-service registry (config 4), one rank simulated "
                      "on one GPU, all-reduces emulated on the GPU",
            "model": args.model, "tp": tp, "services": args.services, "batch": args.batch,
            "steps": args.steps, "engine_steps": len(steps), "plans": plans,
            "emulated_allreduce_calls": sim_ar.calls,
            "measured_step_s": round(compute_s / args.steps, 3),
            "measured_plans_per_s": round(plans / compute_s, 2),
            "p50_latency_ms": round(lats[len(lats) // 2] * 1e3, 1),
            "tp_overlap_min_tokens": model._overlap_min_t if model._comm is not None else None,
            "emulation": "each all-reduce = a kernel holding K12's CUs (its block count) for the "
                         "xGMI model's time (parallel/xgmi_model.py), on the stream the model "
                         "issues it on (the comm stream of the row-chunked MLP block at >= "
                         "tp_overlap_min_tokens tokens, else in line)",
            "data": "synthetic intents, random-init weights"}), flush=True)
        return
    # K12 sizes measured on a grid (64-token steps of [T, H] bf16, up to the K12
    # limit): two processes on this ONE GPU - what that times is mostly the
    # two contexts' time-slicing on one device, not links, so it only backs
    # the pessimistic variant below
    grid = sorted({min(car_max, -(-m // (64 * H * 2)) * 64 * H * 2) for m in msgs if m <= car_max})
    k12 = {b: 0.0 for b in grid}              # CPU dry run: the link model alone
    if grid and cuda and not args.no_k12_timing:
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = free_port()
        procs = [ctx.Process(target=_k12_timer, args=(r, 2, port, grid, q)) for r in range(2)]
        for p in procs:
            p.start()
        got = {}
        try:
            for _ in range(2):
                r, out = q.get(timeout=300)
                got[r] = out
        finally:
            for p in procs:
                p.join(timeout=30)
                if p.is_alive():
                    p.kill()
        if any(isinstance(v, str) for v in got.values()):
            raise RuntimeError(f"K12 timing failed: {got}")
        k12 = {nbytes: max(got[0][nbytes], got[1][nbytes]) for nbytes in grid}

    # the xGMI cost model (parallel/xgmi_model.py) picks and prices each call:
    # the same rule the AllReduce dispatch follows at run time
    comm = {"k12-1": 0.0, "k12-2": 0.0, "rccl": 0.0}
    ncalls = {"k12-1": 0, "k12-2": 0, "rccl": 0}
    pess_s = 0.0
    for m in msgs:
        path, us = xm.best(m, tp, car_max)
        comm[path] += us * 1e-6
        ncalls[path] += 1
        if path.startswith("k12"):
            b = min(car_max, -(-m // (64 * H * 2)) * 64 * H * 2)
            us = max(us, k12.get(b, 0.0))
        pess_s += us * 1e-6
    comm_s = sum(comm.values())
    plans = len(seqs_all)
    pred_s = compute_s + comm_s
    print(json.dumps({
        "config": "llama3-70b TP planner, 50-service registry (config 4), one rank simulated on one GPU",
        "model": args.model, "tp": tp, "services": args.services, "batch": args.batch,
        "steps": args.steps, "engine_steps": len(steps), "tokens": sum(T for T, _ in steps),
        "plans": plans, "graphs_captured": ncap,
        "rank_compute_s": round(compute_s, 3),
        "rank_compute_plans_per_s": round(plans / compute_s, 2),
        "allreduce_calls": ncalls, "allreduce_s": {k: round(v, 3) for k, v in comm.items()},
        "predicted_step_s": round(pred_s / args.steps, 3),
        "predicted_plans_per_s": round(plans / pred_s, 2),
        "predicted_p50_latency_ms_upper": round(lats[len(lats) // 2] * pred_s / compute_s * 1e3, 1),
        "pessimistic_plans_per_s": round(plans / (compute_s + pess_s), 2),
        # NOT implemented - the bound a two-micro-batch schedule could reach
        # (each half's all-reduces under the other half's GEMMs), charging the
        # half-size GEMMs 5 % for their lower efficiency
        "two_microbatch_overlap_bound_plans_per_s": round(plans / max(1.05 * compute_s, comm_s), 2),
        "pessimistic_allreduce_s": round(pess_s, 3),
        "k12_one_gpu_two_process_us": {str(k): round(v, 1) for k, v in k12.items()},
        "measured": "rank-0 compute (GEMM shards, attention on its KV heads, fused-norm "
                    "statistics, sampling, scheduler, hipGraphs)",
        "modelled": {"allreduce": "parallel/xgmi_model.py (K12 one-/two-shot vs RCCL per message)",
                     "xgmi_link_GBps_per_direction": xm.LINK_GBS, "barrier_us": xm.BARRIER_US,
                     "rccl_busbw_GBps": xm.RCCL_BUSBW_GBS, "rccl_latency_us": xm.RCCL_LAT_US,
                     "k12_max_bytes": car_max,
                     "overlap": "none: every all-reduce serialised after its GEMM (pessimistic "
                                "variant: K12 calls at max(model, the one-GPU two-process time))"},
        "data": "synthetic intents, random-init weights",
    }), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--services", type=int, default=50)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--max-nodes", type=int, default=5)
    ap.add_argument("--min-nodes", type=int, default=5,
                    help="min == max fixes the plan size, so the work per plan does not depend on "
                         "the random weights' stop decisions (as bench.py; round 3 ran 1-6 nodes, "
                         "where a random 70B stopped after one)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--seq-parallel", action="store_true",
                    help="Megatron sequence parallelism (reduce-scatter / all-gather) for TP > 1")
    ap.add_argument("--gpus", type=int, default=1, help="TP degree = ranks (one per GPU); N > 1 self-launches")
    ap.add_argument("--no-k12-timing", action="store_true",
                    help="--simulate-rank: skip the two-process K12 timing on this GPU")
    ap.add_argument("--emulate-comm", action="store_true",
                    help="--simulate-rank: run every all-reduce as an emulated K12 call on the GPU "
                         "(measured overlap) instead of pricing it after the run")
    ap.add_argument("--simulate-rank", type=int, default=0, metavar="TP",
                    help="predict config 4 at TP=N from one rank's shards on one GPU (simulate_rank)")
    args = ap.parse_args()
    if args.simulate_rank > 1:
        return simulate_rank(args)
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
    import mcp_amd.planner.grammar as planner_grammar

    eng = LLMEngine(model, num_blocks=nb, max_batch=args.batch + 8, max_step_tokens=16384,
                    temperature=0.2, seed=args.seed, bcast=bcast)
    reg = MemoryRegistry(synthetic_registry(args.services, seed=4))
    planner = LocalPlanner(eng, reg, max_nodes=args.max_nodes, min_nodes=args.min_nodes,
                           retrieval_threshold=10 ** 9)
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
        "tokens": eng.stats["tokens"], "engine_steps": eng.stats["steps"],
        # min_nodes - max_nodes nodes (the random model's stop decisions in between)
        "nodes_per_plan": round(statistics.mean(len(d["nodes"]) for d in dags), 2) if dags else None,
        "plan_view": "compact" if getattr(planner_grammar, "COMPACT", True) else "full",
        "execution": exec_stats,
    }), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
