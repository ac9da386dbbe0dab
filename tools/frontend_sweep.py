"""API front-end throughput sweep on the CPU (no GPU): ``python -m
mcp_amd.api.server`` with MCP_REPLICAS stub replica processes behind the
router (service time 0, plan cache off), for each (front end, API workers)
setting, driven by ``tools/http_load.py`` (closed loop, keep-alive).  Client,
API workers and replicas share this host's CPUs.  One JSON line per setting.

    python tools/frontend_sweep.py [--replicas 8] [--seconds 5] [--conns 32] [--procs 3]
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def start(port: int, http: str, workers: int, replicas: int) -> subprocess.Popen:
    env = dict(os.environ, MCP_PLANNER_BACKEND="local", MCP_MODEL="stub", MCP_REPLICAS=str(replicas),
               MCP_ROUTER="1", MCP_SYNTHETIC_SERVICES="10", MCP_STUB_LATENCY_MS="0",
               MCP_STUB_PLAN_NODES="5", MCP_PLAN_CACHE="0", PYTHONPATH=ROOT)
    p = subprocess.Popen([sys.executable, "-m", "mcp_amd.api.server", "--host", "127.0.0.1",
                          "--port", str(port), "--workers", str(workers), "--http", http,
                          "--no-access-log"],
                         cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL,
                         text=True, start_new_session=True)
    ready, t0 = 0, time.time()
    while ready < workers:
        line = p.stdout.readline()
        if not line:
            raise RuntimeError("server exited during start-up")
        ready += "ready on" in line or "Uvicorn running" in line or "Application startup complete" in line
        if time.time() - t0 > 180:
            raise RuntimeError("server start-up timed out")
    time.sleep(1.0)
    return p


def stop(p: subprocess.Popen):
    try:
        os.killpg(p.pid, signal.SIGTERM)
        p.wait(timeout=60)
    except Exception:  # noqa: BLE001
        os.killpg(p.pid, signal.SIGKILL)
        p.wait(timeout=30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, default=8)
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--conns", type=int, default=32)
    ap.add_argument("--procs", type=int, default=3)
    ap.add_argument("--settings", default="uvicorn:1,fast:1,fast:2,fast:4")
    ap.add_argument("--port", type=int, default=18731)
    a = ap.parse_args()
    for i, st in enumerate(a.settings.split(",")):
        http, workers = st.split(":")
        port = a.port + i
        p = start(port, http, int(workers), a.replicas)
        try:
            out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "http_load.py"), "--port",
                                  str(port), "--seconds", str(a.seconds), "--conns", str(a.conns),
                                  "--procs", str(a.procs)], capture_output=True, text=True, timeout=300)
            rec = json.loads(out.stdout.strip().splitlines()[-1])
        finally:
            stop(p)
        print(json.dumps({"http": http, "api_workers": int(workers), "replicas": a.replicas,
                          "planner": "stub", **rec}), flush=True)


if __name__ == "__main__":
    main()
