"""Loader of the native CPU runtime (``csrc/runtime/runtime.cpp`` ->
``engine/_runtime*.so``, built in-tree by ``csrc/build.py``).

Exports the C++ paged-KV ``BlockAllocator`` (as ``NativeBlockAllocator``),
``pack_step`` (one ragged step's whole int32 descriptor in one host buffer)
and ``topo_generations`` (generational Kahn order).  ``available()`` is False
when the extension was not built; the engine then uses the Python versions in
``kv_cache`` / ``batch`` (same results, checked by tests/test_runtime_cpu.py).
Set ``MCP_NATIVE_RUNTIME=0`` to force the Python versions.
"""
from __future__ import annotations

import glob
import importlib.machinery
import importlib.util
import os

_HERE = os.path.dirname(os.path.abspath(__file__))


def _load():
    if os.environ.get("MCP_NATIVE_RUNTIME", "1") == "0":
        return None
    cands = sorted(glob.glob(os.path.join(_HERE, "_runtime*.so")))
    if not cands:
        return None
    loader = importlib.machinery.ExtensionFileLoader("_runtime", cands[0])
    spec = importlib.util.spec_from_file_location("_runtime", cands[0], loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    return mod


_RT = _load()


def available() -> bool:
    return _RT is not None


def library_path():
    c = sorted(glob.glob(os.path.join(_HERE, "_runtime*.so")))
    return c[0] if c else None


if _RT is not None:
    NativeBlockAllocator = _RT.BlockAllocator
    OutOfBlocks = _RT.OutOfBlocks
    pack_step = _RT.pack_step
    topo_generations = _RT.topo_generations
