#!/usr/bin/env python3
"""Benchmarks for the BASELINE.json configs other than the headline one.

  python bench_suite.py plumbing            # config 1: CPU, stub planner
  python bench_suite.py topk [--n 10000]    # config 3: HBM top-k cosine (GPU)
  python bench_suite.py e2e [--n 10000]     # config 3 end to end: /plan over a 10k registry

Config 1 mirrors the reference measurements in BASELINE.md / SURVEY §6 (stub
LLM, MockTransport services, FastAPI TestClient, p50 of 30 runs):
``/plan`` overhead at 3/10/50/1000 services and ``/execute`` overhead on
3/10/50-node chains.  Each line is JSON.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

REF_PLAN_MS = {3: 1.42, 10: 1.53, 50: 1.81, 1000: 8.79}          # SURVEY §6 (another host)
REF_EXEC_MS = {3: 1.89, 10: 3.16, 50: 10.08}


def load_reference(path: str = "/root/reference/control_plane.py", canned=None):
    """The reference app on THIS host for same-host comparisons:
    a scratch copy of ``control_plane.py`` in a temp dir with only its
    escaped-docstring SyntaxError fixed (D1), imported against stub ``redis`` /
    ``psycopg2`` / ``pgvector`` / ``openai`` modules (an instant LLM returning
    ``canned``).  Nothing of the reference is stored in this repo; returns the
    module (``.app``, ``.orch``) or None when the file is absent."""
    import importlib.util
    import tempfile
    import types
    if not os.path.exists(path):
        return None
    src = open(path, encoding="utf-8").read().replace('\\"\\"\\"', '"""')
    store = {}

    class _Redis:
        def scan_iter(self, pattern):
            pre = pattern.rstrip("*")
            return [k for k in list(store) if k.startswith(pre)]

        def get(self, k):
            return store.get(k)

    reply = json.dumps(canned or {"nodes": [], "edges": []})

    class _Completion:
        @staticmethod
        def create(**kw):
            msg = types.SimpleNamespace(content=reply)
            return types.SimpleNamespace(choices=[types.SimpleNamespace(message=msg)])
    stubs = {"redis": types.SimpleNamespace(from_url=lambda url: _Redis()),
             "psycopg2": types.SimpleNamespace(connect=lambda dsn: object()),
             "pgvector": types.ModuleType("pgvector"),
             "pgvector.psycopg2": types.SimpleNamespace(register_vector=lambda conn: None),
             "openai": types.SimpleNamespace(ChatCompletion=_Completion, api_key=None)}
    saved = {k: sys.modules.get(k) for k in stubs}
    sys.modules.update(stubs)
    try:
        d = tempfile.mkdtemp(prefix="refcp_")
        f = os.path.join(d, "control_plane_scratch.py")
        with open(f, "w", encoding="utf-8") as fh:
            fh.write(src)
        spec = importlib.util.spec_from_file_location("control_plane_scratch", f)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    mod._store = store
    return mod


def _plumbing_cases():
    """Config-1 cases shared by our timing and the reference worker."""
    from mcp_amd.registry import synthetic_registry
    canned = {"nodes": [{"name": "a", "endpoint": "http://a/api", "inputs": {"x": "uid"}}], "edges": []}
    cases = []
    for n in (3, 10, 50, 1000):
        cases.append(("plan", n, synthetic_registry(n, seed=1), lambda i: {"intent": f"charge order {i}"}))
    for n in (3, 10, 50):
        nodes = [{"name": f"n{i}", "endpoint": f"http://n{i}/api",
                  "inputs": {"x": f"n{i - 1}" if i else "uid"}} for i in range(n)]
        edges = [{"from": f"n{i - 1}", "to": f"n{i}"} for i in range(1, n)]
        body = (lambda nodes, edges: lambda i: {"graph": {"nodes": nodes, "edges": edges},
                                               "payload": {"uid": 1}})(nodes, edges)
        cases.append(("execute", n, synthetic_registry(3), body))
    return canned, cases


def _time_posts(c, route, body_fn, k):
    for i in range(5):
        c.post(route, json=body_fn(i))
    ts = []
    for i in range(k):
        t = time.perf_counter()
        r = c.post(route, json=body_fn(i))
        ts.append(time.perf_counter() - t)
        assert r.status_code == 200, r.text
    return statistics.median(ts) * 1e3


def _mock_handler(request):
    import httpx
    return httpx.Response(200, json={"ok": True})


def reference_worker() -> None:
    """Runs in its OWN process (``ReferenceTimer``): loads the scratch copy of
    the reference and answers ``{"case": i, "runs": k}`` lines on stdin with
    the p50 of that case on stdout.  The reference is third-party source: its
    import-time code never runs inside the bench process."""
    import httpx
    from fastapi.testclient import TestClient
    canned, cases = _plumbing_cases()
    ref = load_reference(canned=canned)
    print(json.dumps({"ready": ref is not None}), flush=True)
    if ref is None:
        return
    clients = {}
    for line in sys.stdin:
        req = json.loads(line)
        kind, n, services, body = cases[req["case"]]
        if req["case"] not in clients:
            ref._store.clear()
            for s in services:
                ref._store["mcp:service:" + s["name"]] = json.dumps(dict(s))
            ref.orch.client = httpx.AsyncClient(transport=httpx.MockTransport(_mock_handler))
            clients = {req["case"]: TestClient(ref.app)}
        ms = _time_posts(clients[req["case"]], "/" + kind, body, req["runs"])
        print(json.dumps({"p50_ms": ms}), flush=True)


class ReferenceTimer:
    """The same-host reference comparison, opt-in (``--with-reference``): a
    child ``python -I`` (isolated mode: no user site, no PYTHON* env) in a
    scratch working directory, with a minimal environment, driven over pipes."""

    def __init__(self):
        import subprocess
        import tempfile
        env = {"PATH": os.environ.get("PATH", "/usr/bin:/bin"), "HOME": tempfile.gettempdir()}
        code = ("import sys; sys.path.insert(0, %r); import bench_suite; bench_suite.reference_worker()"
                % os.path.dirname(os.path.abspath(__file__)))
        self.proc = subprocess.Popen([sys.executable, "-I", "-c", code], stdin=subprocess.PIPE,
                                     stdout=subprocess.PIPE, text=True, env=env,
                                     cwd=tempfile.mkdtemp(prefix="refbench_"))
        self.ready = bool(json.loads(self.proc.stdout.readline() or "{}").get("ready"))

    def time(self, case: int, runs: int) -> float:
        self.proc.stdin.write(json.dumps({"case": case, "runs": runs}) + "\n")
        self.proc.stdin.flush()
        return json.loads(self.proc.stdout.readline())["p50_ms"]

    def close(self):
        try:
            self.proc.stdin.close()
            self.proc.wait(timeout=30)
        except Exception:            # noqa: BLE001 - best effort
            self.proc.kill()


def plumbing(runs: int = 30, rounds: int = 3, out=None, with_reference: bool = False):
    """Config 1 on this host.  With ``with_reference`` a stubbed scratch copy
    of the reference runs in an isolated child process (``ReferenceTimer``)
    and the two alternate ``rounds`` times per case, ``runs`` requests each;
    otherwise the reference's recorded numbers (another host) are
    quoted."""
    import httpx
    from fastapi.testclient import TestClient
    from mcp_amd.api.server import create_app
    from mcp_amd.config import Settings
    from mcp_amd.planner.base import StubPlanner
    from mcp_amd.registry import MemoryRegistry

    canned, cases = _plumbing_cases()
    ref = ReferenceTimer() if with_reference else None
    if ref is not None and not ref.ready:
        ref.close()
        ref = None

    def emit(rec):
        line = json.dumps(rec)
        print(line, flush=True)
        if out:
            with open(out, "a") as fh:
                fh.write(line + "\n")

    try:
        for ci, (kind, n, services, body) in enumerate(cases):
            reg = MemoryRegistry(services)
            planner = StubPlanner(reg, canned=canned) if kind == "plan" else StubPlanner(reg)
            app = create_app(Settings(), registry=reg, planner=planner,
                             transport=httpx.MockTransport(_mock_handler))
            o, r = [], []
            with TestClient(app) as c:
                for _ in range(rounds):
                    o.append(_time_posts(c, "/" + kind, body, runs))
                    if ref is not None:
                        r.append(ref.time(ci, runs))
            rec = {"config": f"plumbing/{kind}", ("services" if kind == "plan" else "nodes"): n,
                   "p50_ms": round(statistics.median(o), 3), "rounds_ms": [round(x, 3) for x in o]}
            if r:
                rec.update(reference_same_host_ms=round(statistics.median(r), 3),
                           reference_rounds_ms=[round(x, 3) for x in r],
                           speedup=round(statistics.median(r) / statistics.median(o), 2))
            else:
                rec.update(reference_other_host_ms=(REF_PLAN_MS if kind == "plan" else REF_EXEC_MS)[n])
            emit(rec)
    finally:
        if ref is not None:
            ref.close()


def topk(n: int, dim: int, k: int, batches=(1, 16, 32, 64), iters: int = 50):
    import torch
    import mcp_amd.ops as ops
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    corpus = torch.randn(n, dim, device=dev, generator=g).bfloat16()
    ops.l2norm_rows(corpus)
    for b in batches:
        q = torch.randn(b, dim, device=dev, generator=g).bfloat16()
        ops.l2norm_rows(q)
        v, i = ops.topk_cosine(q, corpus, k)
        # fp32 reference in 1M-row chunks (one [B, 10M] fp32 GEMM through
        # torch.matmul returned wrong scores at 10M x 64 in round 1, see
        # profiles/config3_topk.md), running top-k over the chunks
        qf = q.float()
        rv = None
        for c0 in range(0, n, 1 << 20):
            cs = qf @ corpus[c0:c0 + (1 << 20)].float().t()
            cv, _ = torch.topk(cs, min(k, cs.shape[1]), dim=-1)
            rv = cv if rv is None else torch.topk(torch.cat([rv, cv], 1), k, dim=-1)[0]
            del cs
        # rank check with a tie tolerance: same top-k values, and every
        # returned row really has the returned score (ties may pick another row)
        vdiff = float((v - rv).abs().max())
        direct = (qf.unsqueeze(1) * corpus[i.long()].float()).sum(-1)
        gdiff = float((direct - v).abs().max())
        ok = vdiff <= 1e-4 and gdiff <= 1e-4
        for _ in range(3):
            ops.topk_cosine(q, corpus, k)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            ops.topk_cosine(q, corpus, k)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / iters
        gbs = n * dim * 2 / ms / 1e6
        print(json.dumps({"config": "topk_cosine", "corpus": n, "dim": dim, "k": k, "queries": b,
                          "latency_ms": round(ms, 4), "corpus_GBps": round(gbs, 1), "exact": ok,
                          "max_value_diff": vdiff, "max_gather_diff": gdiff,
                          "path": "fused" if (b <= 64 and k <= 64 and dim in (512, 1024)
                                            and b * n >= ops.FUSED_TOPK_MIN_SCORES) else "gemm+segment"}),
              flush=True)


def e2e(n: int, model: str, runs: int, conc: int, churn: int):
    """Config 3 end to end: ``/plan`` through the FastAPI app with the local
    planner over an ``n``-service registry.  Every request pays retrieval
    (HBM top-k cosine over the schema index), prompt + grammar build,
    tokenisation, prefill + constrained decode and JSON parse.  Three phases:
    one client in a loop, ``conc`` concurrent clients, and ``conc`` clients
    while ``churn`` services are registered in the background (the index
    takes them incrementally, off the engine thread)."""
    import threading

    import httpx
    import torch
    from fastapi.testclient import TestClient
    from mcp_amd.api.server import create_app
    from mcp_amd.config import Settings
    from mcp_amd.planner.local import LocalPlanner
    from mcp_amd.planner.prompt import synthetic_intent
    from mcp_amd.registry import MemoryRegistry, synthetic_registry
    from mcp_amd.utils.metrics import METRICS
    import logging
    logging.getLogger("httpx").setLevel(logging.WARNING)
    cuda = torch.cuda.is_available()
    reg = MemoryRegistry(synthetic_registry(n, seed=3))
    # fixed 5-node plans (min == max, as bench.py / bench_tp.py): the work per
    # request does not depend on the random weights' stop decisions, so the
    # latency spread is the system's, not the plan sizes' (MCP_E2E_NODES)
    nodes = int(os.environ.get("MCP_E2E_NODES", "5"))
    st = Settings(planner_backend="local", model=model, max_batch=max(16, 2 * conc),
                  max_nodes=nodes, min_nodes=nodes, temperature=0.2,
                  kv_blocks=0 if cuda else 1024, topk=int(os.environ.get("MCP_TOPK", "32")))
    t0 = time.perf_counter()
    planner = LocalPlanner.from_settings(st, reg)
    from mcp_amd.utils.heap import settle as settle_heap
    settle_heap()                  # as the server does once it is up
    startup_s = time.perf_counter() - t0
    app = create_app(st, registry=reg, planner=planner,
                     transport=httpx.MockTransport(lambda r: httpx.Response(200, json={})))
    names_seen = set()
    hit = {}

    def client(c, base, k, lats):
        for i in range(k):
            t = time.perf_counter()
            r = c.post("/plan", json={"intent": synthetic_intent(base + i)})
            lats.append(time.perf_counter() - t)
            assert r.status_code == 200, r.text
            names_seen.update(x["name"] for x in r.json()["graph"]["nodes"])

    def blocks():
        st_ = planner.engine.stats
        return st_.get("prefix_blocks", 0), st_.get("prefix_blocks_reused", 0)

    def phase(c, clients, base):
        lats, ths, errs = [], [], []
        b0 = blocks()

        def run(j):
            try:
                client(c, base + j * runs, runs, lats)
            except Exception as e:  # noqa: BLE001 - re-raised below
                errs.append(e)
        t = time.perf_counter()
        for j in range(clients):
            ths.append(threading.Thread(target=run, args=(j,)))
            ths[-1].start()
        for th in ths:
            th.join()
        if errs:
            raise errs[0]
        b1 = blocks()
        nb, nr = b1[0] - b0[0], b1[1] - b0[1]
        # prompt-prefix 64-token blocks this phase needed, and the share found
        # already computed (block-level prefix cache, engine.block_reuse)
        hit.update(prefix_blocks=nb, prefix_blocks_reused=nr,
                   prefix_block_hit_rate=round(nr / nb, 3) if nb else None)
        return lats, time.perf_counter() - t

    def phases(n):
        """p50 / p99 (ms) of the engine-side phases of the phase's last n requests
        (queue: submit -> admitted, ttft: -> first sampled token, decode: the rest)."""
        out = {}
        for k in ("queue_s", "ttft_s", "decode_s"):
            if k in METRICS.windows:
                v = sorted(list(METRICS.windows[k].samples)[-n:])
                if v:
                    out[k[:-2]] = [round(v[len(v) // 2] * 1e3, 1), round(v[min(len(v) - 1, int(len(v) * 0.99))] * 1e3, 1)]
        return out

    def report(name, lats, wall, clients, **extra):
        q = statistics.quantiles(lats, n=100) if len(lats) >= 2 else [lats[0]] * 99
        ret = list(METRICS.windows["retrieval_s"].samples)[-len(lats):] \
            if "retrieval_s" in METRICS.windows else []
        extra = {"phase_p50_p99_ms": phases(len(lats)), **extra}
        print(json.dumps({"config": f"e2e/plan/{name}", "services": n, "model": model,
                          "device": "cuda" if cuda else "cpu", "clients": clients,
                          "requests": len(lats), "p50_ms": round(statistics.median(lats) * 1e3, 2),
                          "p90_ms": round(q[89] * 1e3, 2), "p99_ms": round(q[98] * 1e3, 2),
                          "plans_per_s": round(len(lats) / wall, 2),
                          "retrieval_p50_ms": round(statistics.median(ret) * 1e3, 3) if ret else None,
                          "startup_s": round(startup_s, 1), "topk": st.topk,
                          "nodes_per_plan": [st.min_nodes, st.max_nodes], **hit,
                          "data": "synthetic registry + intents, random-init weights", **extra}),
              flush=True)

    with TestClient(app) as c:
        phase(c, 1, 900_000)                                 # warm the request path
        lats, wall = phase(c, 1, 0)
        report("single", lats, wall, 1)
        lats, wall = phase(c, conc, 100_000)
        report("concurrent", lats, wall, conc)
        if os.environ.get("MCP_E2E_CHURN_PHASE", "1") == "0":     # A/B sweeps: two phases only
            planner._stop.set()
            return
        stop = threading.Event()
        extra = [dict(synthetic_registry(1, seed=10_000 + i)[0]) for i in range(churn)]

        def register():
            for i, rec in enumerate(extra):
                if stop.is_set():
                    break
                rec["name"] = f"late-svc-{i}"
                reg.register(rec)
                time.sleep(0.01)
        th = threading.Thread(target=register)
        th.start()
        lats, wall = phase(c, conc, 200_000)
        stop.set()
        th.join()
        late = {s["name"] for s in reg.list_services() if s["name"].startswith("late-svc-")}
        report("concurrent+registrations", lats, wall, conc, planned_services=len(names_seen),
               registered=len(late),
               index=dict(getattr(planner.retriever, "stats", {})))
    planner._stop.set()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("which", choices=["plumbing", "topk", "e2e"])
    ap.add_argument("--n", type=int, default=10000)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--runs", type=int, default=20, help="e2e: requests per client per phase")
    ap.add_argument("--clients", type=int, default=16, help="e2e: concurrent clients")
    ap.add_argument("--churn", type=int, default=100, help="e2e: services registered during a phase")
    ap.add_argument("--dim", type=int, default=1024)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--out", default=None, help="plumbing: also append the JSON lines here")
    ap.add_argument("--with-reference", action="store_true",
                    help="plumbing: time a stubbed scratch copy of /root/reference/control_plane.py "
                         "in an isolated child process (off by default)")
    a = ap.parse_args()
    if a.which == "plumbing":
        plumbing(out=a.out, with_reference=a.with_reference)
    elif a.which == "e2e":
        e2e(a.n, a.model, a.runs, a.clients, a.churn)
    else:
        topk(a.n, a.dim, a.k)
