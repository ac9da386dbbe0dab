"""HBM-resident schema-embedding store + top-k cosine retrieval.

The reference keeps ``service_schemas(name, input_schema_vector)`` in
PostgreSQL/pgvector and has a fetch helper that is never called
(control_plane.py:46-55).  Here the vectors live in GPU memory
(bf16, unit-norm rows; 10^8 x 1024 fits in 288 GB) and retrieval is the
``ops.topk_cosine`` HIP path (MFMA scoring + segmented top-k).  It bounds the
planner prompt when the registry outgrows the context.

Embeddings: a deterministic signed feature-hashing embedder over word tokens
and character trigrams of the schema text (``ServiceRecord.schema_text``) and
of the intent (native C++ in ``engine/_runtime``, Python fallback with
identical sums).  It needs no model weights and gives lexical similarity,
which is what matching intents to service schemas needs without a trained
encoder.  External vectors can be loaded with ``SchemaIndex.set_vectors``.

The index is incremental, like the reference's persistent table: a registry
change embeds only the records whose schema text changed (upsert by name;
removals swap the last row into the hole), and with ``start_background()``
the diff and the embedding run on a refresher thread.  The thread that owns
the GPU (the engine's scheduler, in ``search``) only applies the finished
updates - an ``index_copy`` of the changed rows - so a registration into a
10k-service registry never stalls the decode loop on a full re-embed.
"""
from __future__ import annotations

import contextlib
import re
import threading
import time
import zlib
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import ops

_WORD = re.compile(r"[a-z0-9]+")


def _hash_embed_sums_py(texts: Sequence[str], dim: int) -> np.ndarray:
    out = np.zeros((len(texts), dim), np.float32)
    for r, t in enumerate(texts):
        t = t.lower().replace("_", " ").replace("-", " ")
        feats = _WORD.findall(t)
        grams = []
        for w in feats:
            ww = f"#{w}#"
            grams += [ww[i:i + 3] for i in range(len(ww) - 2)]
        for f, wgt in [(x, 1.0) for x in feats] + [(g, 0.5) for g in grams]:
            h = zlib.crc32(f.encode())
            out[r, h % dim] += wgt if (h >> 31) & 1 else -wgt
    return out


def _native():
    from ..engine import native
    rt = native._RT if native.available() else None
    return rt if rt is not None and hasattr(rt, "hash_embed_sums") else None


def hash_embed(texts: Sequence[str], dim: int = 1024, native: Optional[bool] = None) -> np.ndarray:
    """Unit-norm [len(texts), dim] float32 feature-hashing embeddings.  ASCII
    texts go through the native embedder (same sums as the Python loop, which
    handles the rest: Unicode lower-casing can map into ASCII)."""
    texts = list(texts)
    rt = _native() if native is not False else None
    if rt is not None and all(t.isascii() for t in texts):
        out = np.asarray(rt.hash_embed_sums(texts, dim))
    elif rt is not None:
        asc = [i for i, t in enumerate(texts) if t.isascii()]
        out = _hash_embed_sums_py([texts[i] if not texts[i].isascii() else "" for i in
                                   range(len(texts))], dim)
        if asc:
            out[asc] = np.asarray(rt.hash_embed_sums([texts[i] for i in asc], dim))
    else:
        out = _hash_embed_sums_py(texts, dim)
    n = np.linalg.norm(out, axis=1, keepdims=True)
    return out / np.maximum(n, 1e-12)


def _text(s) -> str:
    return s.schema_text() if hasattr(s, "schema_text") else str(s)


class _Update:
    """One computed change of the corpus: rows to (over)write with vectors,
    the new row count and the names in row order."""
    __slots__ = ("rows", "vecs", "n", "names", "version")

    def __init__(self, rows, vecs, n, names, version):
        self.rows, self.vecs, self.n, self.names, self.version = rows, vecs, n, names, version


class SchemaIndex:
    def __init__(self, registry=None, dim: int = 1024, device="cpu"):
        self.registry = registry
        self.dim = dim
        self.device = torch.device(device)
        self._version = None
        self.names: List[str] = []
        self.vectors: Optional[torch.Tensor] = None     # [capacity, dim] bf16, unit rows [0, n)
        self.n = 0
        # host shadow of the corpus (the refresher diffs against it): name ->
        # (row, crc of its schema text)
        self._rows: Dict[str, Tuple[int, int]] = {}
        self._shadow_names: List[str] = []
        self._seen: Dict[str, object] = {}               # name -> the record object indexed
        # two locks: ``_diff_lock`` serialises the shadow diffs and their
        # embedding (refresher thread or a synchronous catch-up), ``_lock``
        # only guards the hand-over of finished updates - the engine thread's
        # ``sync`` never waits behind an embedding
        self._lock = threading.Lock()
        self._diff_lock = threading.Lock()
        self._shadow_version = None                     # registry version the shadow reflects
        self._pending: List[_Update] = []
        # a search that finds the registry ahead of the index by at most this
        # many changed records diffs them itself (a service registered just
        # before a /plan is visible to it); larger backlogs stay on the refresher
        self.sync_max_changes = 64
        self._thread: Optional[threading.Thread] = None
        self._stop = threading.Event()
        self.stats = {"embedded": 0, "applied": 0, "full_builds": 0}
        self._by_memo = None                            # see _by_name
        # the index's own GPU stream (non-blocking w.r.t. the default stream
        # the engine's forwards run on): every write and every query of the
        # corpus is ordered on it, and a query's host read-back waits for the
        # top-k kernels only, not behind the engine step queued ahead of it
        self._stream = torch.cuda.Stream(device=self.device) if self.device.type == "cuda" else None

    def _on_stream(self):
        return torch.cuda.stream(self._stream) if self._stream is not None else contextlib.nullcontext()

    # ---------------------------------------------------------- bulk load
    def set_vectors(self, names: Sequence[str], vectors) -> None:
        """Upload and normalise a whole corpus (external vectors).  Rows are
        padded to a multiple of 4 here (zero rows, never returned: ``n_valid``)
        so no query ever copies the corpus (the unfused scoring GEMM writes
        16-B column groups)."""
        with self._on_stream():
            self._set_vectors(names, vectors)

    def _set_vectors(self, names, vectors) -> None:
        v = torch.as_tensor(vectors).to(self.device, torch.bfloat16)
        n = v.shape[0]
        if n % 4:
            v = torch.cat([v, v.new_zeros(4 - n % 4, v.shape[1])])
        v = v.contiguous()
        ops.l2norm_rows(v)
        with self._diff_lock, self._lock:
            self._pending.clear()
            self.names, self.vectors, self.n = list(names), v, n
            self._shadow_names = list(names)
            self._rows = {nm: (i, -1) for i, nm in enumerate(names)}
            self._seen = {}

    # ---------------------------------------------------------- incremental
    def _diff(self, services: Sequence[dict], version) -> Optional[_Update]:
        """CPU side of a refresh (any thread): embed the new / changed records,
        swap-remove the vanished ones; the shadow state moves to the result.
        Caller holds ``self._diff_lock``."""
        want = {}
        for s in services:
            want[s["name"]] = s
        rows, names = self._rows, self._shadow_names
        writes: Dict[int, str] = {}                     # row -> name whose vector goes there
        texts: Dict[str, str] = {}
        # removals: move the last row into each hole
        for nm in [x for x in names if x not in want]:
            self._seen.pop(nm, None)
            r, _ = rows.pop(nm)
            last = len(names) - 1
            if r != last:
                mv = names[last]
                names[r] = mv
                rows[mv] = (r, rows[mv][1])
                writes[r] = mv
            names.pop()
            writes.pop(last, None)
        seen = self._seen
        for nm, s in want.items():
            # a record object already indexed is unchanged (registries hand out
            # the same record objects until a record is re-registered): skip
            # its text and hash - the diff of a 10k registry stays ~1 ms of
            # Python (the GIL is shared with the engine thread)
            cur = rows.get(nm)
            if cur is not None and seen.get(nm) is s:
                continue
            t = _text(s)
            h = zlib.crc32(t.encode("utf-8", "surrogatepass"))
            seen[nm] = s
            if cur is None:
                rows[nm] = (len(names), h)
                writes[len(names)] = nm
                names.append(nm)
            elif cur[1] != h:
                rows[nm] = (cur[0], h)
                writes[cur[0]] = nm
            texts[nm] = t
        if not writes and len(names) == self.n and not self._pending:
            return None
        order = sorted(writes)
        vecs = hash_embed([texts.get(writes[r]) or _text(want[writes[r]]) for r in order], self.dim) \
            if order else np.zeros((0, self.dim), np.float32)
        self.stats["embedded"] += len(order)
        return _Update(np.asarray(order, np.int64), vecs, len(names), list(names), version)

    def _diff_changes(self, changed: Sequence[str], version) -> Optional[_Update]:
        """O(changes) diff from a registry change log (``changes_since``):
        the named records are re-read (``registry.get``) and upserted, or
        swap-removed when gone.  Caller holds ``self._diff_lock``."""
        rows, names = self._rows, self._shadow_names
        writes: Dict[int, str] = {}
        recs: Dict[str, object] = {}
        for nm in changed:
            s = self.registry.get(nm)
            cur = rows.get(nm)
            if s is None:
                if cur is None:
                    continue
                self._seen.pop(nm, None)
                rows.pop(nm)
                r, last = cur[0], len(names) - 1
                if r != last:
                    mv = names[last]
                    names[r] = mv
                    rows[mv] = (r, rows[mv][1])
                    writes[r] = mv
                names.pop()
                writes.pop(last, None)
                continue
            recs[nm] = s
            self._seen[nm] = s
            h = zlib.crc32(_text(s).encode("utf-8", "surrogatepass"))
            if cur is None:
                rows[nm] = (len(names), h)
                writes[len(names)] = nm
                names.append(nm)
            elif cur[1] != h:
                rows[nm] = (cur[0], h)
                writes[cur[0]] = nm
        order = sorted(writes)
        texts = []
        for r in order:
            nm = writes[r]
            s = recs.get(nm) or self._seen.get(nm) or self.registry.get(nm)
            texts.append(_text(s))
        vecs = hash_embed(texts, self.dim) if order else np.zeros((0, self.dim), np.float32)
        self.stats["embedded"] += len(order)
        return _Update(np.asarray(order, np.int64), vecs, len(names), list(names), version)

    def _apply(self, u: _Update) -> None:
        """GPU side (the thread that owns the device): grow the padded
        corpus when needed and write the changed rows."""
        with self._on_stream():
            self._apply_rows(u)

    def _apply_rows(self, u: _Update) -> None:
        cap = 0 if self.vectors is None else self.vectors.shape[0]
        need = -(-max(u.n, 1) // 4) * 4
        if need > cap:
            # headroom: registrations after the first build land in spare rows
            # instead of re-allocating + copying the whole corpus on the engine
            # thread (a synchronous copy on the CPU tier)
            new_cap = max(-(-int(need * 1.25) // 4) * 4, -(-int(cap * 1.5) // 4) * 4, 64)
            nv = torch.zeros(new_cap, self.dim, device=self.device, dtype=torch.bfloat16)
            if self.vectors is not None and self.n:
                nv[:self.n].copy_(self.vectors[:self.n])
            self.vectors = nv
        if len(u.rows):
            v = torch.from_numpy(u.vecs).to(self.device, torch.bfloat16).contiguous()
            ops.l2norm_rows(v)
            self.vectors.index_copy_(0, torch.from_numpy(u.rows).to(self.device), v)
        if u.n < self.n:                                # rows past the end: zero (never returned)
            self.vectors[u.n:self.n].zero_()
        self.n, self.names, self._version = u.n, u.names, u.version
        self.stats["applied"] += 1

    def refresh(self, services: Optional[Sequence[dict]] = None) -> None:
        """Synchronous incremental refresh (diff + apply on this thread)."""
        ver = getattr(self.registry, "version", None)
        if services is None:
            if self.vectors is not None and ver == self._version and not self._pending:
                return
            services = self.registry.list_services()
        with self._diff_lock:
            if self.vectors is None:
                self.stats["full_builds"] += 1
            u = self._diff(services, ver)
            self._shadow_version = ver
            with self._lock:
                pend, self._pending = self._pending, []
        for p in pend:
            self._apply(p)
        if u is not None:
            self._apply(u)
        else:
            self._version = ver

    def sync(self) -> int:
        """Apply the updates the background refresher finished (cheap: the
        changed rows only).  Returns how many were applied."""
        if not self._pending:
            return 0
        with self._lock:
            pend, self._pending = self._pending, []
        for p in pend:
            self._apply(p)
        return len(pend)

    def _catch_up(self, max_changes: Optional[int] = None) -> bool:
        """Bring the shadow up to the registry's current version (diff + embed
        under ``_diff_lock``, then queue the update).  With ``max_changes``
        only a change-log backlog of at most that many records is taken, and
        the call never waits for the lock: the engine thread passes it, and a
        busy lock means the refresher is already diffing (and embedding) a
        backlog, which stays on that thread.  Returns whether the shadow is
        now current."""
        ver = getattr(self.registry, "version", None)
        if ver is None or ver == self._shadow_version:
            return True
        if not self._diff_lock.acquire(blocking=max_changes is None):
            return False
        try:
            seen = self._shadow_version
            ver = getattr(self.registry, "version", None)
            if ver == seen:
                return True
            # a registry with a change log: O(changes); else a full diff
            ch = self.registry.changes_since(seen) \
                if seen is not None and hasattr(self.registry, "changes_since") else None
            if ch is not None:
                if max_changes is not None and len(ch[1]) > max_changes:
                    return False
                ver, names = ch
                u = self._diff_changes(names, ver)
            elif max_changes is not None:
                return False
            else:
                u = self._diff(self.registry.list_services(), ver)
            self._shadow_version = ver
            if u is not None:
                with self._lock:
                    self._pending.append(u)
        finally:
            self._diff_lock.release()
        return True

    def start_background(self, poll_s: float = 0.05) -> None:
        """Refresher thread: watches ``registry.version`` and prepares the
        incremental updates off the engine thread (``sync`` applies them)."""
        if self._thread is not None or self.registry is None:
            return
        if self._shadow_version is None:
            self._shadow_version = self._version

        def loop():
            while not self._stop.wait(poll_s):
                try:
                    self._catch_up()
                except Exception:      # noqa: BLE001 - a registry hiccup: retry next poll
                    time.sleep(poll_s)

        self._thread = threading.Thread(target=loop, name="schema-index-refresh", daemon=True)
        self._thread.start()

    def stop_background(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
            self._thread = None

    # ---------------------------------------------------------- queries
    def embed_queries(self, intents: Sequence[str]) -> torch.Tensor:
        q = torch.from_numpy(hash_embed(intents, self.dim)).to(self.device, torch.bfloat16)
        return ops.l2norm_rows(q.contiguous())

    def search_names(self, intents: Sequence[str], k: int):
        n_pad = -(-self.n // 4) * 4
        with self._on_stream():
            vals, idx = ops.topk_cosine(self.embed_queries(intents), self.vectors[:n_pad], k,
                                        n_valid=self.n)
            idx = idx.cpu().tolist()
            vals = vals.cpu()
        return [[self.names[i] for i in row if 0 <= i < len(self.names)] for row in idx], vals

    def search(self, intent: str, k: int, services: Sequence[dict]) -> List[dict]:
        if self._thread is not None and self.vectors is not None:
            # background mode: a short change-log backlog (a registration
            # just before this request) is diffed here so the request sees
            # it; a large one stays on the refresher thread
            self._catch_up(self.sync_max_changes)
            self.sync()
        elif self.vectors is None or getattr(self.registry, "version", None) != self._version \
                or self.n != len(services):
            self.refresh(services)
        names, _ = self.search_names([intent], k)
        return [s for s in map(self._by_name(services).get, names[0]) if s is not None]

    def _by_name(self, services: Sequence[dict]) -> dict:
        """name -> record of ``services``, memoised on the list's identity:
        its length, its first and last records (held here, so their ids stay
        theirs) and the registry version.  The registry hands out the same
        record objects until it changes, so a 10k-service registry is indexed
        once per version instead of once per request."""
        key = (len(services), id(services[0]) if services else 0,
               id(services[-1]) if services else 0, getattr(self.registry, "version", None))
        memo = self._by_memo
        if memo is None or memo[0] != key:
            memo = self._by_memo = (key, {s["name"]: s for s in services},
                                    (services[0], services[-1]) if services else ())
        return memo[1]
