"""Minimal Redis (RESP2) client and an in-process RESP server.

The reference talks to Redis through ``redis-py`` (control_plane.py:5,28,33-34).
That package is not part of this image, and the GPU boxes have no network, so
the framework ships its own dependency-free RESP2 implementation:

* ``RespClient``  – blocking client with pipelining (``execute_many``), used by
  ``RedisRegistry``.  Supports ``redis://[:password@]host:port/db`` URLs.
* ``RespServer``  – a small threaded server implementing the subset of commands
  the control plane uses (GET/SET/MGET/DEL/SCAN/KEYS/INCR/INCRBY/HINCRBY/
  HINCRBYFLOAT/HGETALL/HSET/PING/SELECT/FLUSHDB/DBSIZE/EXISTS).  It backs
  tests, demos and benchmarks where no Redis binary exists.
"""
from __future__ import annotations

import fnmatch
import socket
import socketserver
import threading
from typing import Dict, List, Optional, Sequence, Tuple
from urllib.parse import urlparse


class RespError(Exception):
    pass


def encode_command(args: Sequence) -> bytes:
    parts = [b"*%d\r\n" % len(args)]
    for a in args:
        if isinstance(a, bytes):
            b = a
        elif isinstance(a, str):
            b = a.encode("utf-8")
        else:
            b = str(a).encode("utf-8")
        parts.append(b"$%d\r\n%s\r\n" % (len(b), b))
    return b"".join(parts)


class _Reader:
    def __init__(self, sock: socket.socket):
        self.sock = sock
        self.buf = bytearray()

    def _fill(self):
        chunk = self.sock.recv(1 << 16)
        if not chunk:
            raise ConnectionError("connection closed by server")
        self.buf += chunk

    def _line(self) -> bytes:
        while True:
            i = self.buf.find(b"\r\n")
            if i >= 0:
                line = bytes(self.buf[:i])
                del self.buf[:i + 2]
                return line
            self._fill()

    def _exact(self, n: int) -> bytes:
        while len(self.buf) < n + 2:
            self._fill()
        data = bytes(self.buf[:n])
        del self.buf[:n + 2]
        return data

    def read(self):
        line = self._line()
        t, rest = line[:1], line[1:]
        if t == b"+":
            return rest.decode()
        if t == b"-":
            return RespError(rest.decode())
        if t == b":":
            return int(rest)
        if t == b"$":
            n = int(rest)
            return None if n < 0 else self._exact(n)
        if t == b"*":
            n = int(rest)
            return None if n < 0 else [self.read() for _ in range(n)]
        raise RespError(f"bad RESP type byte {t!r}")


class RespClient:
    def __init__(self, url: str = "redis://localhost:6379/0", timeout: float = 5.0):
        u = urlparse(url)
        if u.scheme not in ("redis", ""):
            raise ValueError(f"unsupported scheme {u.scheme!r}")
        self.host = u.hostname or "localhost"
        self.port = u.port or 6379
        self.password = u.password
        path = (u.path or "/0").lstrip("/")
        self.db = int(path) if path else 0
        self.timeout = timeout
        self._sock: Optional[socket.socket] = None
        self._reader: Optional[_Reader] = None
        self._lock = threading.Lock()

    # connection is lazy, like redis.from_url (control_plane.py:28)
    def _connect(self):
        s = socket.create_connection((self.host, self.port), timeout=self.timeout)
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._sock, self._reader = s, _Reader(s)
        if self.password:
            self._roundtrip([("AUTH", self.password)])
        if self.db:
            self._roundtrip([("SELECT", self.db)])

    def _roundtrip(self, cmds: List[Tuple]) -> list:
        self._sock.sendall(b"".join(encode_command(c) for c in cmds))
        return [self._reader.read() for _ in cmds]

    def execute_many(self, cmds: List[Tuple]) -> list:
        """Pipeline: one write, N replies.  Errors are returned, not raised."""
        with self._lock:
            if self._sock is None:
                self._connect()
            try:
                return self._roundtrip(cmds)
            except (ConnectionError, OSError):
                self.close()
                self._connect()
                return self._roundtrip(cmds)

    def execute(self, *args):
        r = self.execute_many([tuple(args)])[0]
        if isinstance(r, RespError):
            raise r
        return r

    def close(self):
        if self._sock is not None:
            try:
                self._sock.close()
            finally:
                self._sock = self._reader = None

    # helpers
    def scan_iter(self, match: str, count: int = 1000):
        cursor = b"0"
        while True:
            cursor, keys = self.execute("SCAN", cursor, "MATCH", match, "COUNT", count)
            for k in keys:
                yield k
            if cursor in (b"0", "0", 0):
                return

    def get(self, key):
        return self.execute("GET", key)

    def set(self, key, value):
        return self.execute("SET", key, value)

    def mget(self, keys):
        return self.execute("MGET", *keys) if keys else []

    def delete(self, *keys):
        return self.execute("DEL", *keys) if keys else 0


# ----------------------------------------------------------------------------------
# in-process server
# ----------------------------------------------------------------------------------

def _b(x) -> bytes:
    return x if isinstance(x, bytes) else str(x).encode()


def _encode_reply(v) -> bytes:
    if v is None:
        return b"$-1\r\n"
    if isinstance(v, RespError):
        return b"-" + str(v).encode() + b"\r\n"
    if isinstance(v, bool):
        return b":%d\r\n" % int(v)
    if isinstance(v, int):
        return b":%d\r\n" % v
    if isinstance(v, _Status):
        return b"+" + v.encode() + b"\r\n"
    if isinstance(v, (list, tuple)):
        return b"*%d\r\n" % len(v) + b"".join(_encode_reply(x) for x in v)
    b = _b(v)
    return b"$%d\r\n%s\r\n" % (len(b), b)


class _Status(str):
    pass


OK = _Status("OK")


class _Store:
    def __init__(self):
        self.dbs: Dict[int, Dict[bytes, object]] = {}
        self.lock = threading.Lock()

    def db(self, i: int) -> Dict[bytes, object]:
        return self.dbs.setdefault(i, {})


class _Handler(socketserver.StreamRequestHandler):
    def handle(self):
        store: _Store = self.server.store  # type: ignore[attr-defined]
        reader = _Reader(self.request)
        dbi = 0
        while True:
            try:
                cmd = reader.read()
            except (ConnectionError, OSError):
                return
            if not isinstance(cmd, list) or not cmd:
                return
            name = cmd[0].decode().upper()
            args = cmd[1:]
            try:
                with store.lock:
                    if name == "SELECT":
                        dbi = int(args[0])
                        reply = OK
                    else:
                        reply = self._dispatch(name, args, store.db(dbi))
            except Exception as e:  # noqa: BLE001 - surface as RESP error
                reply = RespError(f"ERR {e}")
            self.request.sendall(_encode_reply(reply))

    @staticmethod
    def _dispatch(name, args, db):
        if name == "PING":
            return _Status("PONG")
        if name == "AUTH":
            return OK
        if name == "GET":
            v = db.get(args[0])
            return v if (v is None or isinstance(v, bytes)) else RespError("WRONGTYPE")
        if name == "SET":
            db[args[0]] = args[1]
            return OK
        if name == "MGET":
            return [db.get(k) if isinstance(db.get(k), bytes) else None for k in args]
        if name == "DEL":
            return sum(1 for k in args if db.pop(k, None) is not None)
        if name == "EXISTS":
            return sum(1 for k in args if k in db)
        if name == "DBSIZE":
            return len(db)
        if name == "FLUSHDB":
            db.clear()
            return OK
        if name in ("KEYS", "SCAN"):
            if name == "KEYS":
                pat = args[0].decode()
                return [k for k in db if fnmatch.fnmatchcase(k.decode(), pat)]
            cursor = int(args[0])
            pat, count = "*", 10
            i = 1
            while i < len(args):
                opt = args[i].decode().upper()
                if opt == "MATCH":
                    pat = args[i + 1].decode()
                elif opt == "COUNT":
                    count = int(args[i + 1])
                i += 2
            keys = sorted(db.keys())
            chunk = keys[cursor:cursor + count]
            nxt = cursor + count if cursor + count < len(keys) else 0
            return [str(nxt).encode(), [k for k in chunk if fnmatch.fnmatchcase(k.decode(), pat)]]
        if name in ("INCR", "INCRBY"):
            by = int(args[1]) if name == "INCRBY" else 1
            v = int(db.get(args[0], b"0")) + by
            db[args[0]] = str(v).encode()
            return v
        if name == "HSET":
            h = db.setdefault(args[0], {})
            new = 0
            for f, v in zip(args[1::2], args[2::2]):
                new += f not in h
                h[f] = v
            return new
        if name == "HINCRBY":
            h = db.setdefault(args[0], {})
            v = int(h.get(args[1], b"0")) + int(args[2])
            h[args[1]] = str(v).encode()
            return v
        if name == "HINCRBYFLOAT":
            h = db.setdefault(args[0], {})
            v = float(h.get(args[1], b"0")) + float(args[2])
            h[args[1]] = repr(v).encode()
            return repr(v).encode()
        if name == "HGETALL":
            h = db.get(args[0], {})
            out = []
            for f, v in h.items():
                out += [f, v]
            return out
        return RespError(f"ERR unknown command '{name}'")


class _TCPServer(socketserver.ThreadingTCPServer):
    allow_reuse_address = True
    daemon_threads = True


class RespServer:
    """``with RespServer() as url: ...`` – an ephemeral Redis-compatible server."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0):
        self._srv = _TCPServer((host, port), _Handler)
        self._srv.store = _Store()  # type: ignore[attr-defined]
        self._thread = threading.Thread(target=self._srv.serve_forever, daemon=True)

    @property
    def url(self) -> str:
        h, p = self._srv.server_address[:2]
        return f"redis://{h}:{p}/0"

    def start(self) -> "RespServer":
        self._thread.start()
        return self

    def stop(self):
        self._srv.shutdown()
        self._srv.server_close()

    def __enter__(self):
        self.start()
        return self.url

    def __exit__(self, *exc):
        self.stop()
