"""Closed-loop HTTP/1.1 load generator for the API front end: ``conns``
keep-alive connections per process, each posting ``/plan`` bodies back to
back; ``procs`` processes.  A raw asyncio client (pre-built request bytes,
Content-Length framing), so the client side costs far less CPU per request
than the server it measures.

    python tools/http_load.py --port 8000 --seconds 5 --conns 32 --procs 2

Prints one JSON line: requests, wall seconds, requests/s, status counts,
p50 / p99 latency (ms).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import multiprocessing as mp
import time


def _request(host: str, port: int, path: str, body: bytes) -> bytes:
    return (f"POST {path} HTTP/1.1\r\nHost: {host}:{port}\r\nContent-Type: application/json\r\n"
            f"Content-Length: {len(body)}\r\n\r\n").encode() + body


async def _conn(host, port, reqs, t_end, lat, status):
    r, w = await asyncio.open_connection(host, port)
    i = 0
    try:
        while time.perf_counter() < t_end:
            t0 = time.perf_counter()
            w.write(reqs[i % len(reqs)])
            i += 1
            head = await r.readuntil(b"\r\n\r\n")
            line_end = head.find(b"\r\n")
            code = int(head[9:12])
            clen = 0
            for h in head[line_end + 2:].split(b"\r\n"):
                if h[:15].lower() == b"content-length:":
                    clen = int(h[15:])
            if clen:
                await r.readexactly(clen)
            lat.append(time.perf_counter() - t0)
            status[code] = status.get(code, 0) + 1
    finally:
        w.close()


async def _run(host, port, path, conns, seconds, nbodies):
    reqs = [_request(host, port, path, json.dumps({"intent": f"charge order {i} and notify"}).encode())
            for i in range(nbodies)]
    lat, status = [], {}
    t0 = time.perf_counter()
    await asyncio.gather(*[_conn(host, port, reqs, t0 + seconds, lat, status) for _ in range(conns)])
    return lat, status, time.perf_counter() - t0


def _proc(args, q):
    lat, status, wall = asyncio.run(_run(args.host, args.port, args.path, args.conns, args.seconds,
                                         args.bodies))
    q.put((lat, status, wall))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--path", default="/plan")
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--conns", type=int, default=32, help="connections per process")
    ap.add_argument("--procs", type=int, default=2)
    ap.add_argument("--bodies", type=int, default=64, help="distinct request bodies")
    args = ap.parse_args(argv)
    q = mp.get_context("fork").Queue()
    ps = [mp.get_context("fork").Process(target=_proc, args=(args, q)) for _ in range(args.procs)]
    for p in ps:
        p.start()
    res = []
    deadline = time.monotonic() + args.seconds + 60
    while len(res) < len(ps):
        try:
            res.append(q.get(timeout=1.0))
        except Exception:               # noqa: BLE001 - queue.Empty
            if time.monotonic() > deadline or any(p.exitcode not in (None, 0) for p in ps):
                for p in ps:
                    p.kill()
                raise SystemExit("load client failed (server down?)")
    for p in ps:
        p.join()
    lat = sorted(x for r in res for x in r[0])
    status = {}
    for r in res:
        for k, v in r[1].items():
            status[k] = status.get(k, 0) + v
    wall = max(r[2] for r in res)
    out = {"requests": len(lat), "wall_s": round(wall, 3), "rps": round(len(lat) / wall, 1),
           "status": status,
           "p50_ms": round(lat[len(lat) // 2] * 1e3, 2) if lat else None,
           "p99_ms": round(lat[int(len(lat) * 0.99)] * 1e3, 2) if lat else None}
    print(json.dumps(out), flush=True)
    return out


if __name__ == "__main__":
    main()
