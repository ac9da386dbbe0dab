"""Open-loop HTTP/1.1 load generator for soak runs of the API (config 5
through the deployment path).

Why not httpx: ``httpx.AsyncClient`` (httpcore 1.0.9 here) re-plans its whole
connection pool on every request start and finish
(``AsyncConnectionPool._assign_requests_to_connections``).  That pass walks
every pooled connection and, for each idle one, counts the idle connections
again: O(C^2) per request with C pooled connections.  At a steady 120
intents/s with ~20 requests in flight C stays small; a stall that lets a few
hundred requests pile up grows the pool to hundreds of connections, and from
then on each request costs the client tens of ms of CPU - the client can no
longer keep pace, requests pile up further, and the run never recovers
(``profiles/soak_root_cause_r6.md`` has the measurement).  Worse, the same
pass walks every *queued* request and, for each, every connection: O(R x C)
per request with R requests waiting in the pool, which is what a backlog
makes large.

This client keeps per-request work O(1): a LIFO stack of idle keep-alive
connections (a new connection only when none is idle, at most
``max_conns``; beyond that requests wait in a FIFO), pre-encoded request
heads, Content-Length framing, no per-request objects beyond the coroutine.
Each request's latency runs from its *scheduled* Poisson arrival, so client
lateness is charged to the measurement, not hidden.  ``progress`` is called
every ``log_s`` seconds - through the drain too - with the window's sent /
done / errors, requests in flight, open connections, the client's own event
loop lag and its GC pauses.
"""
from __future__ import annotations

import asyncio
import collections
import json
import time
from typing import Callable, List, Optional

import numpy as np

from .procstats import GCWatch, LoopLag, rss_mb


class _Conn:
    __slots__ = ("r", "w")

    def __init__(self, r, w):
        self.r, self.w = r, w


class OpenLoopClient:
    def __init__(self, host: str, port: int, max_conns: int = 2048):
        self.host, self.port = host, port
        self.max_conns = max_conns
        self.idle: List[_Conn] = []
        self.nconns = 0
        self.waiters: collections.deque = collections.deque()
        self._hosthdr = f"Host: {host}:{port}\r\n".encode()

    async def _get(self) -> _Conn:
        if self.idle:
            return self.idle.pop()
        if self.nconns < self.max_conns:
            self.nconns += 1
            try:
                r, w = await asyncio.open_connection(self.host, self.port)
            except BaseException:
                self.nconns -= 1
                raise
            return _Conn(r, w)
        fut = asyncio.get_running_loop().create_future()
        self.waiters.append(fut)
        return await fut

    def _put(self, c: _Conn):
        while self.waiters:
            fut = self.waiters.popleft()
            if not fut.done():
                fut.set_result(c)
                return
        self.idle.append(c)

    def _drop(self, c: _Conn):
        self.nconns -= 1
        try:
            c.w.close()
        except Exception:  # noqa: BLE001
            pass

    async def request(self, method: str, path: str, body: bytes = b"") -> tuple:
        """(status, body bytes)."""
        head = (f"{method} {path} HTTP/1.1\r\n").encode() + self._hosthdr
        if body or method == "POST":
            head += b"Content-Type: application/json\r\nContent-Length: %d\r\n" % len(body)
        data = head + b"\r\n" + body
        c = await self._get()
        try:
            c.w.write(data)
            hd = await c.r.readuntil(b"\r\n\r\n")
            status = int(hd[9:12])
            clen = 0
            close = False
            for h in hd.split(b"\r\n")[1:]:
                k, _, v = h.partition(b":")
                k = k.strip().lower()
                if k == b"content-length":
                    clen = int(v)
                elif k == b"connection" and v.strip().lower() == b"close":
                    close = True
            out = await c.r.readexactly(clen) if clen else b""
        except BaseException:
            self._drop(c)
            raise
        if close:
            self._drop(c)
        else:
            self._put(c)
        return status, out

    async def aclose(self):
        for c in self.idle:
            self._drop(c)
        self.idle = []


async def open_loop(host: str, port: int, qps: float, duration: float,
                    body_fn: Callable[[int], bytes], path: str = "/plan", seed: int = 0,
                    log_s: float = 30.0, progress: Optional[Callable[[dict], None]] = None,
                    keep_bodies: bool = True, max_conns: int = 2048,
                    drain_timeout: float = 600.0) -> dict:
    """Poisson arrivals of ``qps``/s for ``duration`` s, then drain.  Returns
    latencies (s, from scheduled arrival), status counts, response bodies
    (``keep_bodies``), the first errors and the per-window log."""
    cl = OpenLoopClient(host, port, max_conns=max_conns)
    rng = np.random.default_rng(seed)
    n = max(1, int(qps * duration))
    arrivals = np.cumsum(rng.exponential(1.0 / qps, n))
    lat = np.full(n, np.nan)
    status = collections.Counter()
    bodies: List[bytes] = [] if keep_bodies else None
    errors: List[str] = []
    st = {"sent": 0, "done": 0, "inflight": 0, "win_sent": 0, "win_done": 0, "win_err": 0,
          "win_inflight_max": 0}
    all_done = asyncio.Event()
    live = set()
    windows: List[dict] = []
    gcw, lag = GCWatch(), LoopLag().start()
    t0 = time.perf_counter()

    async def one(i: int):
        try:
            code, out = await cl.request("POST", path, body_fn(i))
            lat[i] = time.perf_counter() - (t0 + arrivals[i])
            status[code] += 1
            if code != 200:
                st["win_err"] += 1
                if len(errors) < 20:
                    errors.append(f"{code}: {out[:300]!r}")
            elif bodies is not None:
                bodies.append(out)
        except Exception as e:  # noqa: BLE001
            status["exc"] += 1
            st["win_err"] += 1
            if len(errors) < 20:
                errors.append(repr(e))
        finally:
            st["done"] += 1
            st["win_done"] += 1
            st["inflight"] -= 1
            if st["done"] == n:
                all_done.set()

    async def reporter():
        t_last = t0
        while True:
            await asyncio.sleep(log_s)
            now = time.perf_counter()
            win = now - t_last
            t_last = now
            rec = {"t": round(now - t0, 1), "sent": st["sent"], "done": st["done"], "of": n,
                   "sent_per_s": round(st["win_sent"] / win, 1),
                   "done_per_s": round(st["win_done"] / win, 1), "errors": st["win_err"],
                   "inflight": st["inflight"], "inflight_max": st["win_inflight_max"],
                   "conns": cl.nconns, "idle_conns": len(cl.idle),
                   "rss_mb": round(rss_mb(), 1)}
            rec.update(lag.snapshot())
            rec.update(gcw.snapshot())
            st["win_sent"] = st["win_done"] = st["win_err"] = 0
            st["win_inflight_max"] = st["inflight"]
            windows.append(rec)
            if progress is not None:
                progress(rec)

    rep = asyncio.get_running_loop().create_task(reporter())
    try:
        for i in range(n):
            delay = t0 + arrivals[i] - time.perf_counter()
            if delay > 0:
                await asyncio.sleep(delay)
            st["sent"] += 1
            st["win_sent"] += 1
            st["inflight"] += 1
            if st["inflight"] > st["win_inflight_max"]:
                st["win_inflight_max"] = st["inflight"]
            task = asyncio.ensure_future(one(i))
            live.add(task)                   # the loop holds tasks weakly
            task.add_done_callback(live.discard)
        t_sent = time.perf_counter()
        await asyncio.wait_for(all_done.wait(), drain_timeout)
        elapsed = time.perf_counter() - t0
    finally:
        rep.cancel()
        lag.stop()
        gcw.close()
        await cl.aclose()
    ok = lat[~np.isnan(lat)]
    return {"n": n, "elapsed_s": elapsed, "send_s": t_sent - t0, "latencies": ok,
            "status": dict(status), "bodies": bodies, "errors": errors, "windows": windows}


def plan_body(intent: str) -> bytes:
    return json.dumps({"intent": intent}).encode()
