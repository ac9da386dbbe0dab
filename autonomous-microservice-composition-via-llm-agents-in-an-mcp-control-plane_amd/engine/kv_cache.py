"""Paged KV cache resident in HBM + block allocator with prefix sharing.

Layout (one allocation): ``[layers, 2(K|V), num_blocks, kv_heads/tp, 64, head_dim]``
bf16.  A block holds one 64-key attention tile of one kv head contiguously
(16 KiB at head_dim 128), which is exactly what ``csrc/attention.hip`` stages
with 16 LDS-DMA wave-instructions.  Sized from free HBM (288 GB per MI355X):
Llama-3-8B needs 128 KiB per token, so ~200 GB holds ~1.6 M tokens.

Blocks are reference counted so many requests can share the registry-prompt
prefix blocks (prefix caching).
"""
from __future__ import annotations

from typing import List, Optional

import torch

from . import native
from .batch import BLOCK_SIZE

if native.available():
    OutOfBlocks = native.OutOfBlocks
else:
    class OutOfBlocks(RuntimeError):
        pass


class BlockAllocator:
    """Free-list allocator with refcounts.  The engine uses the C++ one
    (``native.NativeBlockAllocator``, csrc/runtime/runtime.cpp) when built;
    this is the reference implementation and CPU fallback."""

    def __init__(self, num_blocks: int):
        self.num_blocks = num_blocks
        self._free: List[int] = list(range(num_blocks - 1, -1, -1))
        self._ref = [0] * num_blocks

    @property
    def num_free(self) -> int:
        return len(self._free)

    def alloc(self, n: int) -> List[int]:
        if n > len(self._free):
            raise OutOfBlocks(f"need {n} KV blocks, {len(self._free)} free")
        out = [self._free.pop() for _ in range(n)]
        for b in out:
            self._ref[b] = 1
        return out

    def incref(self, blocks: List[int]):
        for b in blocks:
            if self._ref[b] <= 0:
                raise RuntimeError(f"incref of free block {b}")
            self._ref[b] += 1

    def free(self, blocks: List[int]):
        for b in blocks:
            if self._ref[b] <= 0:
                raise RuntimeError(f"double free of block {b}")
            self._ref[b] -= 1
            if self._ref[b] == 0:
                self._free.append(b)

    def refcount(self, b: int) -> int:
        return self._ref[b]

    def utilization(self) -> float:
        return 1.0 - len(self._free) / max(1, self.num_blocks)


def make_allocator(num_blocks: int):
    if native.available():
        return native.NativeBlockAllocator(num_blocks)
    return BlockAllocator(num_blocks)


class KVCache:
    def __init__(self, layers: int, kv_heads: int, head_dim: int, num_blocks: int, device,
                 dtype=torch.bfloat16):
        self.layers, self.kv_heads, self.head_dim = layers, kv_heads, head_dim
        self.num_blocks = num_blocks
        self.data = torch.zeros(layers, 2, num_blocks, kv_heads, BLOCK_SIZE, head_dim,
                                device=device, dtype=dtype)
        self.allocator = make_allocator(num_blocks)

    def layer(self, l: int):
        return self.data[l, 0], self.data[l, 1]

    @staticmethod
    def bytes_per_block(layers, kv_heads, head_dim, dtype_bytes=2) -> int:
        return layers * 2 * kv_heads * BLOCK_SIZE * head_dim * dtype_bytes

    @classmethod
    def sized_for(cls, layers, kv_heads, head_dim, device, budget_bytes: Optional[int] = None,
                  max_blocks: Optional[int] = None, reserve_frac: float = 0.1):
        per = cls.bytes_per_block(layers, kv_heads, head_dim)
        dev = torch.device(device)
        if budget_bytes is None:
            if dev.type == "cuda":
                free, total = torch.cuda.mem_get_info(dev)
                budget_bytes = int(free - reserve_frac * total)
            else:
                budget_bytes = 256 * per
        n = max(16, budget_bytes // per)
        if max_blocks is not None:
            n = min(n, max_blocks)
        return cls(layers, kv_heads, head_dim, int(n), device)
