"""Cost model of the tensor-parallel all-reduce paths on one MI355X node
(VERDICT r4 weak #5 / next #3d): which of K12 one-shot, K12
two-shot and RCCL to use for a message of ``m`` bytes over ``n`` ranks.

Topology: every GPU has one xGMI link to each of the 7 others (the task
statement's 7 x ~153 GB/s per GPU, bidirectional: ~76.8 GB/s per link and
direction).  K12 (csrc/custom_allreduce.hip) reads peers' IPC-mapped staging
buffers directly, so the n - 1 peer reads of one phase run on n - 1 links at
once:

* one-shot: stage (local copy) + 1 flag barrier + read the whole message from
  each peer (one link each): ``m / link``;
* two-shot: stage + 2 barriers + reduce-scatter (a 1/n slice from each peer)
  + all-gather (the reduced 1/n slice of each peer): ``2 m / (n link)``;
* RCCL ring: ``2 (n - 1) / n * m / busbw`` plus a fixed latency, busbw at
  most (n - 1) links (one ring per link).

Constants are environment-overridable (``MCP_XGMI_*``); they are datasheet /
topology figures, not measurements - no multi-GPU box was available to this
build (the one-GPU K12 timings of two processes on one device measure process
time-slicing, not links; bench_tp.py reports both).  Crossovers at the
defaults: one-shot beats two-shot below ~307 KB at n = 8 (~461 KB at n = 4;
always at n = 2: two-shot moves the same bytes with one more barrier); K12
two-shot beats RCCL at every size (a lower intercept and a lower slope: reads
on all 7 links at once vs. a ring), so K12 takes every message its staging
buffer holds and RCCL only the rest.
"""
from __future__ import annotations

import os


def _f(name: str, default: float) -> float:
    return float(os.environ.get(name, str(default)))


LINK_GBS = _f("MCP_XGMI_LINK_GBS", 76.8)          # per link and direction
BARRIER_US = _f("MCP_XGMI_BARRIER_US", 3.0)       # one cross-GPU flag barrier
LAUNCH_US = _f("MCP_XGMI_LAUNCH_US", 1.5)         # a kernel boundary
STAGE_GBS = _f("MCP_XGMI_STAGE_GBS", 4000.0)      # local HBM copy into staging (read + write)
RCCL_BUSBW_GBS = _f("MCP_XGMI_RCCL_BUSBW_GBS", 300.0)
RCCL_LAT_US = _f("MCP_XGMI_RCCL_LAT_US", 25.0)


def _us(nbytes: float, gbs: float) -> float:
    return nbytes / (gbs * 1e3)                    # GB/s = 1e3 bytes per us


def one_shot_us(m: int, n: int) -> float:
    return LAUNCH_US + _us(m, STAGE_GBS) + BARRIER_US + _us(m, LINK_GBS)


def two_shot_us(m: int, n: int) -> float:
    return LAUNCH_US + _us(m, STAGE_GBS) + 2 * BARRIER_US + 2 * _us(m / n, LINK_GBS)


def rccl_us(m: int, n: int) -> float:
    # a ring uses one link per GPU and direction; with n - 1 links to the
    # group's peers RCCL can run at most n - 1 rings
    busbw = min(RCCL_BUSBW_GBS, (n - 1) * LINK_GBS)
    return RCCL_LAT_US + _us(2 * (n - 1) / n * m, busbw)


def k12_mode(m: int, n: int) -> int:
    """1 (one-shot) or 2 (two-shot), whichever the model prices lower."""
    return 1 if one_shot_us(m, n) <= two_shot_us(m, n) else 2


def best(m: int, n: int, k12_max_bytes: int):
    """(path, modelled us): "k12-1" / "k12-2" (message fits the staging
    buffer) or "rccl"."""
    opts = [("rccl", rccl_us(m, n))]
    if m <= k12_max_bytes:
        opts += [("k12-1", one_shot_us(m, n)), ("k12-2", two_shot_us(m, n))]
    return min(opts, key=lambda o: o[1])


def one_shot_max_bytes(n: int, hi: int = 1 << 30) -> int:
    """Largest message the model sends one-shot at ``n`` ranks (binary search
    on the monotone crossover; ``hi`` when one-shot always wins)."""
    if k12_mode(hi, n) == 1:
        return hi
    lo_b, hi_b = 0, hi
    while hi_b - lo_b > 16:
        mid = (lo_b + hi_b) // 2
        if k12_mode(mid, n) == 1:
            lo_b = mid
        else:
            hi_b = mid
    return lo_b
