"""Per-process health statistics for long serving runs.

The reference has no instrumentation at all (control_plane.py:90-91 configures
logging only).  A control plane that must hold a steady request rate for
hours needs to show, per process and per time window, where time goes when it
falls behind.  This module gathers the cheap, always-valid signals:

* ``GCWatch``   - cyclic-GC pauses (count, total and max ms per generation)
  through ``gc.callbacks``;
* ``LoopLag``   - asyncio event-loop lag: a ticker that asks to wake every
  ``period`` seconds and records how late it actually woke;
* ``rss_mb()``  - resident set size from ``/proc/self/statm``;
* ``StatsLog``  - appends one JSON line per window to a file (``MCP_STATS_FILE``)
  or stderr.

Each ``snapshot()`` returns the window since the previous snapshot and resets
it, so a log line always describes the last window only.
"""
from __future__ import annotations

import asyncio
import gc
import json
import os
import sys
import threading
import time
from typing import Callable, Optional


def rss_mb() -> float:
    try:
        with open("/proc/self/statm") as f:
            return int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE") / 2 ** 20
    except (OSError, ValueError, IndexError):
        return 0.0


class GCWatch:
    """Cyclic-collector pauses since the last ``snapshot()``."""

    def __init__(self):
        self._t0 = 0.0
        self._gen = 0
        self._lock = threading.Lock()
        self._reset()
        gc.callbacks.append(self._cb)

    def _reset(self):
        self.count = [0, 0, 0]
        self.total_ms = [0.0, 0.0, 0.0]
        self.max_ms = 0.0

    def _cb(self, phase, info):
        if phase == "start":
            self._t0 = time.perf_counter()
            self._gen = info.get("generation", 0)
            return
        dt = (time.perf_counter() - self._t0) * 1e3
        g = min(2, self._gen)
        with self._lock:
            self.count[g] += 1
            self.total_ms[g] += dt
            self.max_ms = max(self.max_ms, dt)

    def snapshot(self) -> dict:
        with self._lock:
            out = {"gc_count": list(self.count), "gc_ms": [round(x, 1) for x in self.total_ms],
                   "gc_max_ms": round(self.max_ms, 1)}
            self._reset()
        return out

    def close(self):
        try:
            gc.callbacks.remove(self._cb)
        except ValueError:
            pass


class LoopLag:
    """Event-loop lag: how late a ``period``-second ticker wakes up."""

    def __init__(self, period: float = 0.05):
        self.period = period
        self._task: Optional[asyncio.Task] = None
        self._reset()

    def _reset(self):
        self.n = 0
        self.sum = 0.0
        self.max = 0.0

    def start(self, loop: Optional[asyncio.AbstractEventLoop] = None):
        loop = loop or asyncio.get_running_loop()
        self._task = loop.create_task(self._tick())
        return self

    async def _tick(self):
        while True:
            t = time.perf_counter()
            await asyncio.sleep(self.period)
            lag = time.perf_counter() - t - self.period
            self.n += 1
            self.sum += lag
            if lag > self.max:
                self.max = lag

    def snapshot(self) -> dict:
        out = {"loop_lag_mean_ms": round(1e3 * self.sum / max(1, self.n), 2),
               "loop_lag_max_ms": round(1e3 * self.max, 1)}
        self._reset()
        return out

    def stop(self):
        if self._task is not None:
            self._task.cancel()


class StatsLog:
    """One JSON line per window: to ``path`` (appended, flushed per line) or stderr."""

    def __init__(self, path: Optional[str] = None):
        self.path = path
        self._lock = threading.Lock()

    def write(self, rec: dict):
        line = json.dumps(rec, separators=(",", ":"))
        with self._lock:
            if self.path:
                with open(self.path, "a") as f:
                    f.write(line + "\n")
            else:
                print(line, file=sys.stderr, flush=True)


def stats_period() -> float:
    """``MCP_STATS_S``: seconds per stats window (0 = off)."""
    try:
        return float(os.environ.get("MCP_STATS_S", "0") or 0)
    except ValueError:
        return 0.0


async def report_forever(period: float, snap: Callable[[], dict], log: StatsLog,
                         proc: str):
    """Write ``snap()`` plus the GC / loop / RSS window every ``period`` s (the
    coroutine of a serving process's stats task; cancel it to stop)."""
    gcw = GCWatch()
    lag = LoopLag().start()
    t_start = time.time()

    def report(final: bool = False):
        rec = {"proc": proc, "pid": os.getpid(), "t": round(time.time() - t_start, 1),
               "rss_mb": round(rss_mb(), 1)}
        if final:
            rec["final"] = True             # the partial window up to shutdown
        rec.update(lag.snapshot())
        rec.update(gcw.snapshot())
        try:
            rec.update(snap())
        except Exception as e:  # noqa: BLE001 - stats must never take the server down
            rec["snap_error"] = repr(e)
        log.write(rec)

    try:
        while True:
            await asyncio.sleep(period)
            report()
    except asyncio.CancelledError:
        report(final=True)                  # every request of the run is in some line
        raise
    finally:
        lag.stop()
        gcw.close()
