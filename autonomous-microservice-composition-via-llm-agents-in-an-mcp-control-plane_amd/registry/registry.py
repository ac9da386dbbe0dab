"""Service registry backends.

Reference: ``ServiceRegistry.list_services`` (control_plane.py:26-35) does
``SCAN MATCH mcp:service:*`` followed by one ``GET`` per key (N+1 round trips),
in arbitrary SCAN order, and crashes with ``json.loads(None)`` when a key is
deleted between SCAN and GET.

Here:
* the key prefix and record schema are identical (T1);
* ``RedisRegistry`` pipelines the reads (SCAN pages + one MGET per page), skips
  vanished keys and returns records **sorted by name** so prompts are
  deterministic;
* ``MemoryRegistry`` is a drop-in in-process backend;
* both expose ``version`` (bumped on every write) so the planner can cache
  prompt prefixes / embeddings keyed by registry version;
* telemetry counters (README.md:43-44 claims Prometheus -> Redis telemetry that
  the reference never implemented) are recorded with ``record_call``.
"""
from __future__ import annotations

import threading
from typing import Dict, Iterable, List, Optional

from ..config import SERVICES_PREFIX, TELEMETRY_PREFIX
from .records import ServiceRecord
from .resp import RespClient, RespError


class BaseRegistry:
    prefix: str = SERVICES_PREFIX

    def list_services(self) -> List[ServiceRecord]:
        raise NotImplementedError

    def register(self, rec) -> None:
        raise NotImplementedError

    def unregister(self, name: str) -> bool:
        raise NotImplementedError

    @property
    def version(self) -> int:
        raise NotImplementedError

    def register_many(self, recs: Iterable) -> None:
        for r in recs:
            self.register(r)

    def get(self, name: str) -> Optional[ServiceRecord]:
        for s in self.list_services():
            if s.name == name:
                return s
        return None

    # telemetry -------------------------------------------------------------
    def record_call(self, name: str, latency_s: float, ok: bool) -> None:  # pragma: no cover - default no-op
        pass

    def telemetry(self, name: str) -> Dict[str, float]:
        return {}


class MemoryRegistry(BaseRegistry):
    CHANGELOG = 65536          # (version, name) entries kept for changes_since

    def __init__(self, records: Iterable = (), prefix: str = SERVICES_PREFIX):
        import collections
        self.prefix = prefix
        self._recs: Dict[str, ServiceRecord] = {}
        self._tel: Dict[str, Dict[str, float]] = {}
        self._version = 0
        self._lock = threading.Lock()
        self._sorted: Optional[List[ServiceRecord]] = None
        self._log = collections.deque(maxlen=self.CHANGELOG)
        self.register_many(records)

    def register(self, rec) -> None:
        rec = ServiceRecord.parse(rec) if not isinstance(rec, ServiceRecord) else rec
        with self._lock:
            self._recs[rec.name] = rec
            self._version += 1
            self._log.append((self._version, rec.name))
            self._sorted = None

    def unregister(self, name: str) -> bool:
        with self._lock:
            ok = self._recs.pop(name, None) is not None
            if ok:
                self._version += 1
                self._log.append((self._version, name))
                self._sorted = None
            return ok

    def changes_since(self, version: int):
        """(current version, names registered / re-registered / removed after
        ``version``) - O(changes), for incremental consumers (the schema
        index); None when the change log no longer reaches back that far."""
        with self._lock:
            cur = self._version
            if version == cur:
                return cur, []
            if not self._log or self._log[0][0] > version + 1:
                return None
            return cur, list({nm: None for v, nm in self._log if v > version})

    def list_services(self) -> List[ServiceRecord]:
        with self._lock:
            if self._sorted is None:
                self._sorted = [self._recs[k] for k in sorted(self._recs)]
            return list(self._sorted)

    def get(self, name: str) -> Optional[ServiceRecord]:
        return self._recs.get(name)

    @property
    def version(self) -> int:
        return self._version

    def record_call(self, name: str, latency_s: float, ok: bool) -> None:
        with self._lock:
            t = self._tel.setdefault(name, {"calls": 0, "errors": 0, "latency_sum": 0.0})
            t["calls"] += 1
            t["errors"] += 0 if ok else 1
            t["latency_sum"] += latency_s

    def telemetry(self, name: str) -> Dict[str, float]:
        return dict(self._tel.get(name, {}))


class RedisRegistry(BaseRegistry):
    VERSION_KEY = "mcp:registry:version"

    def __init__(self, url: str, prefix: str = SERVICES_PREFIX, scan_count: int = 1000):
        self.client = RespClient(url)
        self.prefix = prefix
        self.scan_count = scan_count
        self._cache_version = None
        self._cache: List[ServiceRecord] = []

    def _scan_keys(self) -> List[bytes]:
        return list(self.client.scan_iter(self.prefix + "*", count=self.scan_count))

    def list_services(self) -> List[ServiceRecord]:
        keys = self._scan_keys()
        out: List[ServiceRecord] = []
        # one MGET per page of keys instead of N GETs
        for i in range(0, len(keys), 512):
            page = keys[i:i + 512]
            for raw in self.client.mget(page):
                if raw is None:          # deleted between SCAN and MGET (D12)
                    continue
                try:
                    out.append(ServiceRecord.parse(raw))
                except ValueError:
                    continue
        out.sort(key=lambda r: r.name)
        return out

    def register(self, rec) -> None:
        rec = ServiceRecord.parse(rec) if not isinstance(rec, ServiceRecord) else rec
        self.client.execute_many([("SET", self.prefix + rec.name, rec.dumps()),
                                  ("INCR", self.VERSION_KEY)])

    def register_many(self, recs: Iterable) -> None:
        cmds = []
        for r in recs:
            r = ServiceRecord.parse(r) if not isinstance(r, ServiceRecord) else r
            cmds.append(("SET", self.prefix + r.name, r.dumps()))
        if cmds:
            cmds.append(("INCR", self.VERSION_KEY))
            for rep in self.client.execute_many(cmds):
                if isinstance(rep, RespError):
                    raise rep

    def unregister(self, name: str) -> bool:
        n, _ = self.client.execute_many([("DEL", self.prefix + name), ("INCR", self.VERSION_KEY)])
        return bool(n)

    @property
    def version(self) -> int:
        v = self.client.get(self.VERSION_KEY)
        return int(v) if v is not None else 0

    def record_call(self, name: str, latency_s: float, ok: bool) -> None:
        key = TELEMETRY_PREFIX + name
        self.client.execute_many([("HINCRBY", key, "calls", 1),
                                  ("HINCRBY", key, "errors", 0 if ok else 1),
                                  ("HINCRBYFLOAT", key, "latency_sum", f"{latency_s:.6f}")])

    def telemetry(self, name: str) -> Dict[str, float]:
        flat = self.client.execute("HGETALL", TELEMETRY_PREFIX + name) or []
        return {flat[i].decode(): float(flat[i + 1]) for i in range(0, len(flat), 2)}


def make_registry(redis_url: Optional[str], prefix: str = SERVICES_PREFIX) -> BaseRegistry:
    if redis_url:
        return RedisRegistry(redis_url, prefix=prefix)
    return MemoryRegistry(prefix=prefix)
