#!/usr/bin/env python3
"""Serving benchmarks (BASELINE.json configs 2 and 5).

* ``single`` (config 2): Llama-3-8B TP=1, 10-service registry, ONE intent at a
  time, intent -> DAG latency.  Reported twice: with the registry prompt's
  prefix KV cached (the steady state of a server whose registry did not change)
  and cold (registry prefix recomputed for every intent).
* ``qps`` (config 5): open-loop Poisson arrivals at a fixed rate per GPU into
  the continuously-batching engine (requests join and leave the running batch
  every step; small steps replay captured hipGraphs).  Reports achieved
  plans/s, p50 / p99 intent -> DAG latency (arrival to DAG) and batch stats.
  ``--gpus N`` starts N ranks itself (parallel.launch; or run it under
  torchrun): every rank serves ``--qps`` on its own replica (data parallel),
  the JSON line aggregates the node (plans/s summed, p50 / p99 over every
  rank's requests).

Synthetic intents, random-init weights (no checkpoints offline).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import mcp_amd  # noqa: E402,F401
from mcp_amd.engine.engine import LLMEngine  # noqa: E402
from mcp_amd.models.llama import LlamaModel  # noqa: E402
from mcp_amd.orchestrator import validate_dag  # noqa: E402
from mcp_amd.planner.local import LocalPlanner  # noqa: E402
from mcp_amd.planner.prompt import synthetic_intent  # noqa: E402
from mcp_amd.registry import MemoryRegistry, synthetic_registry  # noqa: E402


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pct(xs, q):
    return float(np.percentile(np.asarray(xs), q)) if xs else float("nan")


def run_single(planner, n, warm):
    lat = []
    for i in range(n):
        t = time.perf_counter()
        planner.plan_many([synthetic_intent(10_000 + i)], fresh_prefix=not warm)
        lat.append(time.perf_counter() - t)
    return lat


def run_qps(planner, engine, qps, duration, seed, rank):
    rng = np.random.default_rng(seed + 7919 * rank)
    n = max(1, int(qps * duration))
    arrivals = np.cumsum(rng.exponential(1.0 / qps, n))
    services = planner.registry.list_services()
    lat, dags = [], []
    done_at = {}
    t0 = time.perf_counter()
    i = 0
    batch_sizes = []
    next_log = 30.0            # a progress line every 30 s (long soak runs stay visibly alive)
    def pump():
        """Submit the arrivals that are due (also the engine's arrival pump
        while it holds a lookahead launch)."""
        nonlocal i
        now = time.perf_counter() - t0
        k = 0
        while i < n and arrivals[i] <= now:
            dec, ptoks, stoks = planner.prepare(synthetic_intent(rank * 1_000_000 + i), services)
            arr = arrivals[i]

            def on_done(seq, arr=arr):
                done_at[seq.uid] = (time.perf_counter() - t0, arr, seq.result)
            engine.submit(dec, stoks, prefix_tokens=ptoks, on_done=on_done)
            i += 1
            k += 1
        return k

    engine.poll_arrivals = pump
    while i < n or engine.has_work():
        now = time.perf_counter() - t0
        if now >= next_log:
            log(f"[qps {qps}] {now:.0f} s: {i} of {n} submitted, {len(done_at)} done, "
                f"{len(engine.running)} running")
            next_log += 30.0
        pump()
        if engine.has_work():
            batch_sizes.append(len(engine.running))
            engine.step()
        elif i < n:
            time.sleep(max(0.0, min(arrivals[i] - (time.perf_counter() - t0), 0.002)))
    elapsed = time.perf_counter() - t0
    engine.poll_arrivals = None
    for t_done, arr, res in done_at.values():
        lat.append(t_done - arr)
        dags.append(res)
    return lat, dags, elapsed, n, batch_sizes


def run_via_api(args):
    """Config 5 through the deployment path: ``python -m mcp_amd.api.server``
    (``--http fast``: the lean HTTP/1.1 front end, or uvicorn + FastAPI;
    ``create_app`` from the environment; ``--api-workers``) in a child
    process with the local planner - ``--replicas N`` DP replica processes
    behind the router (``MCP_REPLICAS`` / ``MCP_ROUTER``), or with
    ``--replicas 0`` the in-process engine thread of a one-GPU server - and
    this process as the load generator: Poisson arrivals of ``--qps`` per
    replica over HTTP (127.0.0.1), each request's time from its scheduled
    arrival to its DAG.  Same model, registry, DAG size and engine limits as
    the direct ``qps`` mode, so the two lines compare the engine with and
    without the front end.

    ``--client raw`` (default): ``utils/loadgen.py``, O(1) client work per
    request; ``--client httpx``: the round-5 httpx client, whose pool costs
    O(connections^2) per request (the cause of the round-5 soak collapse,
    ``profiles/soak_root_cause_r6.md``).  ``--model stub`` runs stub replicas
    (no GPU) with ``--stub-latency-ms`` of service time; ``--stub-stall
    AT:SECONDS`` freezes each replica once.  Every ``--log-s`` seconds, send
    phase and drain alike, the client logs its window (sent / done / in
    flight / loop lag / GC) and the server writes its own (front end, router
    queues, each replica's steps and GC) to ``--stats-file``."""
    import asyncio
    import logging
    import subprocess
    from mcp_amd.parallel.launch import free_port
    from mcp_amd.utils.loadgen import open_loop, plan_body
    logging.getLogger("httpx").setLevel(logging.WARNING)
    port = free_port()
    nrep = max(0, args.replicas)
    env = dict(os.environ, MCP_PLANNER_BACKEND="local", MCP_MODEL=args.model,
               MCP_MAX_BATCH="512", MCP_MAX_STEP_TOKENS="16384", MCP_TEMPERATURE="0.2",
               MCP_MAX_NODES=str(args.max_nodes), MCP_MIN_NODES=str(args.min_nodes),
               MCP_SEED=str(args.seed), MCP_REPLICAS=str(max(1, nrep)),
               MCP_ROUTER="1" if nrep >= 1 else "0", MCP_SYNTHETIC_SERVICES=str(args.services),
               MCP_STATS_S=str(args.log_s))
    if args.stats_file:
        os.makedirs(os.path.dirname(os.path.abspath(args.stats_file)), exist_ok=True)
        open(args.stats_file, "w").close()
        env["MCP_STATS_FILE"] = os.path.abspath(args.stats_file)
    if args.model == "stub":
        env.update(MCP_STUB_LATENCY_MS=str(args.stub_latency_ms),
                   MCP_STUB_PLAN_NODES=str(args.max_nodes))
        if args.stub_stall:
            env["MCP_STUB_STALL"] = args.stub_stall
    if args.no_graphs:
        env["MCP_GRAPHS"] = "0"
    log_path = os.environ.get("MCP_SERVER_LOG", "/tmp/mcp_api_server.log")
    srv = subprocess.Popen([sys.executable, "-m", "mcp_amd.api.server", "--host", "127.0.0.1",
                            "--port", str(port), "--no-access-log", "--http", args.http,
                            "--workers", str(args.api_workers)],
                           env=env, stdout=open(log_path, "w"), stderr=subprocess.STDOUT,
                           cwd=os.path.dirname(os.path.abspath(__file__)))
    reg = MemoryRegistry(synthetic_registry(args.services, seed=1))
    names = [s.name for s in reg.list_services()]
    qps = args.qps * max(1, nrep)

    def progress(rec):
        log(f"[via-api qps {qps} {args.client}] " + json.dumps(rec, separators=(",", ":")))

    async def wait_ready():
        import httpx
        async with httpx.AsyncClient(base_url=f"http://127.0.0.1:{port}", timeout=600.0) as c:
            t0 = time.time()
            while True:                                  # start-up: model init + graph capture
                if srv.poll() is not None:
                    raise RuntimeError(f"server exited ({srv.returncode}); see {log_path}")
                try:
                    if (await c.get("/healthz")).status_code == 200:
                        break
                except httpx.TransportError:
                    pass
                if time.time() - t0 > 900:
                    raise TimeoutError("server did not start")
                await asyncio.sleep(1.0)
            log(f"server ready after {time.time() - t0:.1f}s")
            # the server's in-memory registry holds the same synthetic services
            # (MCP_SYNTHETIC_SERVICES, seed 1)
            await asyncio.gather(*[c.post("/plan", json={"intent": synthetic_intent(-1 - i)})
                                   for i in range(max(1, args.warmup))])

    async def drive_raw():
        await wait_ready()
        res = await open_loop("127.0.0.1", port, qps, args.duration,
                              lambda i: plan_body(synthetic_intent(i)), seed=args.seed,
                              log_s=args.log_s, progress=progress)
        dags = [json.loads(b)["graph"] for b in res["bodies"]]
        errs = res["errors"] if len(res["latencies"]) < res["n"] else []
        import httpx
        async with httpx.AsyncClient(base_url=f"http://127.0.0.1:{port}", timeout=60.0) as c:
            server_metrics["text"] = (await c.get("/metrics")).text
        return list(res["latencies"]), dags, errs, res["elapsed_s"], res["n"], res["windows"]

    async def drive_httpx():
        # the round-5 load generator (kept for the A/B): httpx pool, every
        # task kept; progress now logged through the drain as well
        import httpx
        await wait_ready()
        limits = httpx.Limits(max_connections=4096, max_keepalive_connections=1024)
        async with httpx.AsyncClient(base_url=f"http://127.0.0.1:{port}", timeout=600.0,
                                     limits=limits) as c:
            rng = np.random.default_rng(args.seed)
            n = max(1, int(qps * args.duration))
            arrivals = np.cumsum(rng.exponential(1.0 / qps, n))
            lat, dags, errs = [], [], []
            st = {"sent": 0, "win_done": 0, "win_sent": 0}
            windows = []

            async def one(i):
                try:
                    r = await c.post("/plan", json={"intent": synthetic_intent(i)})
                    if r.status_code != 200:
                        errs.append(r.text)
                        return
                    dags.append(r.json()["graph"])
                    lat.append(time.perf_counter() - (t_start + arrivals[i]))
                finally:
                    st["win_done"] += 1

            async def reporter():
                from mcp_amd.utils.procstats import GCWatch, LoopLag
                gcw, lag = GCWatch(), LoopLag().start()
                t_last = time.perf_counter()
                try:
                    while True:
                        await asyncio.sleep(args.log_s)
                        now = time.perf_counter()
                        win, t_last = now - t_last, now
                        pool = c._transport._pool
                        rec = {"t": round(now - t_start, 1), "sent": st["sent"], "done": len(lat),
                               "of": n, "sent_per_s": round(st["win_sent"] / win, 1),
                               "done_per_s": round(st["win_done"] / win, 1), "errors": len(errs),
                               "inflight": st["sent"] - len(lat) - len(errs),
                               "conns": len(pool.connections)}
                        rec.update(lag.snapshot())
                        rec.update(gcw.snapshot())
                        st["win_done"] = st["win_sent"] = 0
                        windows.append(rec)
                        progress(rec)
                finally:
                    lag.stop()
                    gcw.close()
            tasks = []
            t_start = time.perf_counter()
            rep = asyncio.get_running_loop().create_task(reporter())
            for i in range(n):
                delay = t_start + arrivals[i] - time.perf_counter()
                if delay > 0:
                    await asyncio.sleep(delay)
                tasks.append(asyncio.create_task(one(i)))
                st["sent"] += 1
                st["win_sent"] += 1
            await asyncio.gather(*tasks)
            rep.cancel()
            return lat, dags, errs, time.perf_counter() - t_start, n, windows

    server_metrics = {}
    try:
        lat, dags, errs, elapsed, n, windows = asyncio.run(
            drive_raw() if args.client == "raw" else drive_httpx())
    finally:
        srv.terminate()
        try:
            srv.wait(timeout=60)
        except subprocess.TimeoutExpired:
            srv.kill()
    if errs:
        raise RuntimeError(f"{len(errs)} requests failed: {errs[0][:300]}")
    for d in dags:
        validate_dag(d, names)
    # steady state: windows that ended while arrivals were still being sent
    send_w = [w for w in windows if w["t"] <= args.duration]
    out = {"metric": "plans/sec at fixed QPS through the API (config 5, deployment path)",
           "path": (f"{'fast HTTP/1.1 front end' if args.http == 'fast' else 'uvicorn + FastAPI'}"
                    f" x {args.api_workers} API worker(s) + "
                    f"{'router -> %d replica process(es)' % nrep if nrep else 'in-process engine thread'}"),
           "client": args.client,
           "model": args.model, "services": args.services, "dtype": "bf16",
           "data": "synthetic intents, random-init weights", "replicas": nrep,
           "nodes_per_plan": [args.min_nodes, args.max_nodes], "offered_qps": qps,
           "value": round(len(lat) / elapsed, 2), "unit": "plans/s",
           "p50_latency_ms": round(statistics.median(lat) * 1e3, 1),
           "p99_latency_ms": round(pct(lat, 99) * 1e3, 1), "requests": n, "duration_s": args.duration,
           "window_s": args.log_s,
           "window_done_per_s_min": min((w["done_per_s"] for w in send_w[1:]), default=None),
           "window_done_per_s_max": max((w["done_per_s"] for w in send_w[1:]), default=None),
           "max_inflight": max((w["inflight"] for w in windows), default=None),
           "client_loop_lag_max_ms": max((w["loop_lag_max_ms"] for w in windows), default=None)}
    if server_metrics:
        # the node's own view (replica engines' windows, last 4096 requests
        # each): submit -> DAG inside the engine, and its phases, p50 in ms
        ph = {}
        for ln in server_metrics["text"].splitlines():
            if ln.startswith("mcp_") and 'quantile="0.5"' in ln:
                k = ln.split("{")[0][4:]
                if k in ("plan_latency_s", "queue_s", "ttft_s", "decode_s", "engine_latency_s"):
                    ph[k] = round(float(ln.split()[-1]) * 1e3, 1)
        out["server_p50_ms"] = ph
    if args.model == "stub":
        out.update(dtype=None, data="synthetic intents, stub replicas (no model)",
                   stub_latency_ms=args.stub_latency_ms, stub_stall=args.stub_stall)
    print(json.dumps(out), flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["single", "qps"])
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--services", type=int, default=10)
    ap.add_argument("--n", type=int, default=20, help="single: intents per measurement")
    ap.add_argument("--qps", type=float, default=20.0, help="qps: arrival rate per GPU")
    ap.add_argument("--duration", type=float, default=20.0)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--min-nodes", type=int, default=5)
    ap.add_argument("--max-nodes", type=int, default=5)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU); N > 1 self-launches")
    ap.add_argument("--via-api", action="store_true",
                    help="qps: drive the HTTP API server (child process) instead of the engine")
    ap.add_argument("--replicas", type=int, default=1,
                    help="--via-api: DP replica processes behind the router (0: in-process engine)")
    ap.add_argument("--http", choices=["fast", "uvicorn"], default="fast",
                    help="--via-api: the server's front end")
    ap.add_argument("--api-workers", type=int, default=1,
                    help="--via-api: API worker processes (each routes to its slice of the replicas)")
    ap.add_argument("--client", choices=["raw", "httpx"], default="raw",
                    help="--via-api: load generator (raw: O(1) per request; httpx: round 5's)")
    ap.add_argument("--log-s", type=float, default=30.0,
                    help="--via-api: progress / server stats window, seconds")
    ap.add_argument("--stats-file", default=None,
                    help="--via-api: server-side stats lines (JSONL; default: server log)")
    ap.add_argument("--stub-latency-ms", type=float, default=150.0,
                    help="--via-api --model stub: replica service time per intent")
    ap.add_argument("--stub-stall", default="",
                    help="--via-api --model stub: AT:SECONDS, each replica freezes once")
    args = ap.parse_args()
    if args.via_api:
        return run_via_api(args)
    from mcp_amd.parallel.launch import check_devices, self_launch
    rc = self_launch(args.gpus)
    if rc is not None:
        sys.exit(rc)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    check_devices(int(os.environ.get("LOCAL_WORLD_SIZE", str(world))), local_rank)
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    model = LlamaModel.random(args.model, dev, seed=args.seed)
    engine = LLMEngine(model, max_batch=512, max_step_tokens=16384, temperature=0.2,
                       seed=args.seed + rank, graphs=False if args.no_graphs else None)
    reg = MemoryRegistry(synthetic_registry(args.services, seed=1))
    names = [s.name for s in reg.list_services()]
    planner = LocalPlanner(engine, reg, max_nodes=args.max_nodes, min_nodes=args.min_nodes)
    t_w = time.perf_counter()
    ncap = engine.warm_graphs(contexts=(2048,))            # server start-up: capture the buckets
    warm_s = time.perf_counter() - t_w
    planner.plan_many([synthetic_intent(-1 - i) for i in range(max(1, args.warmup))])
    from mcp_amd.utils.heap import settle as settle_heap
    settle_heap()                                          # as the server does after start-up

    out = {"n_gpus": world, "model": args.model, "services": args.services, "dtype": "bf16",
           "data": "synthetic intents, random-init weights",
           "nodes_per_plan": [args.min_nodes, args.max_nodes]}
    if args.mode == "single":
        run_single(planner, args.warmup, warm=True)         # warms the hipGraph buckets too
        warm = run_single(planner, args.n, warm=True)
        cold = run_single(planner, args.n, warm=False)
        out.update(metric="single-intent intent->DAG latency (config 2)",
                   p50_warm_prefix_ms=round(statistics.median(warm) * 1e3, 2),
                   p90_warm_prefix_ms=round(pct(warm, 90) * 1e3, 2),
                   p50_cold_prefix_ms=round(statistics.median(cold) * 1e3, 2),
                   graph_steps=engine.stats["graph_steps"], steps=engine.stats["steps"],
                   host_us_per_step={k: round(1e6 * engine.stats[k] / max(1, engine.stats["steps"]), 1)
                                     for k in ("schedule_s", "launch_s", "sample_s", "update_s")},
                   replay_host_us_per_graph_step=round(
                       1e6 * engine.graphs.replay_host_s / max(1, engine.graphs.replays), 1)
                   if engine.graphs is not None else None)
    else:
        if world > 1:
            dist.barrier()
        from mcp_amd.utils.metrics import METRICS
        METRICS.reset()
        lat, dags, elapsed, n, bs = run_qps(planner, engine, args.qps, args.duration, args.seed, rank)
        for d in dags:
            validate_dag(d, names)
        mine = {"rate": len(lat) / elapsed, "lat": lat, "bs": float(np.mean(bs)) if bs else 0.0}
        every = [None] * world
        if world > 1:
            dist.all_gather_object(every, mine)
        else:
            every = [mine]
        all_lat = [x for e in every for x in e["lat"]]
        plans_s = sum(e["rate"] for e in every)
        p50, p99 = statistics.median(all_lat), pct(all_lat, 99)
        mean_b = sum(e["bs"] for e in every) / world
        out.update(metric="plans/sec at fixed QPS (config 5)", offered_qps=args.qps * world,
                   value=round(plans_s, 2), unit="plans/s", p50_latency_ms=round(p50 * 1e3, 1),
                   p99_latency_ms=round(p99 * 1e3, 1), mean_running_batch=round(mean_b, 1),
                   graph_steps=engine.stats["graph_steps"], steps=engine.stats["steps"],
                   graph_captures_startup=ncap, graph_warm_s=round(warm_s, 2),
                   graph_captures_total=engine.stats.get("graph_captures", 0),
                   duration_s=args.duration,
                   # per-request phases on this rank, p50 in ms
                   phases_p50_ms={k: round(METRICS.windows[k].quantile(0.5) * 1e3, 3)
                                  for k in ("retrieval_s", "prompt_s", "queue_s", "ttft_s",
                                            "decode_s", "parse_s") if k in METRICS.windows})
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
