"""roctx ranges around engine phases.

``span("engine.schedule")`` pushes a roctx range (``torch.cuda.nvtx`` is the
roctx binding on ROCm builds of PyTorch) when ``MCP_ROCTX=1``, so
``rocprofv3 --marker-trace`` shows the host phases next to the kernels; it is a
no-op otherwise (no overhead on the hot path).
"""
from __future__ import annotations

import contextlib
import os

_ON = os.environ.get("MCP_ROCTX", "0") == "1"


def enabled() -> bool:
    return _ON


@contextlib.contextmanager
def _range(name: str):
    import torch
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()


def span(name: str):
    return _range(name) if _ON else contextlib.nullcontext()
