"""Process-wide metrics with Prometheus text exposition.

The reference only configures logging (control_plane.py:90-91); README.md:43-44
claims Prometheus telemetry that has no code.  This module is dependency-free
(``prometheus_client`` is optional) and backs ``GET /metrics``: plans/sec,
intent->DAG latency quantiles, TTFT, decode tokens/s, batch occupancy,
KV-block utilisation, per-service latency/error counters.
"""
from __future__ import annotations

import bisect
import threading
import time
from collections import defaultdict, deque
from typing import Dict


class _Window:
    """Bounded sample window for quantiles."""

    def __init__(self, maxlen: int = 4096):
        self.samples = deque(maxlen=maxlen)
        self.count = 0
        self.total = 0.0

    def add(self, v: float):
        self.samples.append(v)
        self.count += 1
        self.total += v

    def quantile(self, q: float) -> float:
        if not self.samples:
            return 0.0
        s = sorted(self.samples)
        return s[min(len(s) - 1, int(q * (len(s) - 1) + 0.5))]


class Metrics:
    def __init__(self):
        self._lock = threading.Lock()
        self.counters: Dict[str, float] = defaultdict(float)
        self.gauges: Dict[str, float] = {}
        self.windows: Dict[str, _Window] = defaultdict(_Window)
        self.svc_calls: Dict[str, int] = defaultdict(int)
        self.svc_errors: Dict[str, int] = defaultdict(int)
        self.svc_latency: Dict[str, float] = defaultdict(float)
        self._plan_times = deque(maxlen=100000)
        self.started = time.time()

    def inc(self, name: str, v: float = 1.0):
        with self._lock:
            self.counters[name] += v

    def set(self, name: str, v: float):
        with self._lock:
            self.gauges[name] = v

    def observe(self, name: str, v: float):
        with self._lock:
            self.windows[name].add(v)

    def plan_done(self, latency_s: float):
        now = time.time()
        with self._lock:
            self.counters["plans_total"] += 1
            self.windows["plan_latency_s"].add(latency_s)
            self._plan_times.append(now)

    def plans_per_sec(self, window_s: float = 10.0) -> float:
        now = time.time()
        with self._lock:
            i = bisect.bisect_left(self._plan_times, now - window_s)
            n = len(self._plan_times) - i
        return n / window_s

    def observe_service(self, name: str, latency_s: float, ok: bool):
        with self._lock:
            self.svc_calls[name] += 1
            self.svc_latency[name] += latency_s
            if not ok:
                self.svc_errors[name] += 1

    def reset(self):
        self.__init__()

    def render(self) -> str:
        lines = []
        with self._lock:
            for k, v in sorted(self.counters.items()):
                lines += [f"# TYPE mcp_{k} counter", f"mcp_{k} {v}"]
            for k, v in sorted(self.gauges.items()):
                lines += [f"# TYPE mcp_{k} gauge", f"mcp_{k} {v}"]
            for k, w in sorted(self.windows.items()):
                lines.append(f"# TYPE mcp_{k} summary")
                for q in (0.5, 0.9, 0.99):
                    lines.append(f'mcp_{k}{{quantile="{q}"}} {w.quantile(q)}')
                lines += [f"mcp_{k}_sum {w.total}", f"mcp_{k}_count {w.count}"]
            if self.svc_calls:
                lines.append("# TYPE mcp_service_calls_total counter")
                for n, c in sorted(self.svc_calls.items()):
                    lines.append(f'mcp_service_calls_total{{service="{n}"}} {c}')
                lines.append("# TYPE mcp_service_errors_total counter")
                for n in sorted(self.svc_calls):
                    lines.append(f'mcp_service_errors_total{{service="{n}"}} {self.svc_errors.get(n, 0)}')
                lines.append("# TYPE mcp_service_latency_seconds_sum counter")
                for n, s in sorted(self.svc_latency.items()):
                    lines.append(f'mcp_service_latency_seconds_sum{{service="{n}"}} {s}')
        lines += ["# TYPE mcp_plans_per_second gauge", f"mcp_plans_per_second {self.plans_per_sec()}"]
        return "\n".join(lines) + "\n"


METRICS = Metrics()
