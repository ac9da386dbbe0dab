"""Tensor-parallel serving: one driver rank + (tp - 1) worker ranks.

The driver (TP rank 0) owns the scheduler, block allocator, grammar state and
sampling; every step it broadcasts the packed step descriptor
(``engine.batch.pack_host``) and all ranks run the same sharded forward, whose
row-parallel projections all-reduce over RCCL/xGMI (models.llama).  Workers
hold identical KV-cache layouts (same block count), so block ids in the
descriptor are valid everywhere.  Only the driver samples: after the final
all-reduce every rank has the full hidden state and the LM head is replicated.
Steps that fit a captured bucket are replayed from hipGraphs on every rank
(engine.graphs: the driver broadcasts the graph key, then the static payload).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .. import ops
from ..parallel.comm import StepBroadcaster
from .batch import views


def agree_num_blocks(kv_bytes_per_block: int, device, group, reserve_frac: float = 0.1,
                     cap: int = None) -> int:
    """All TP ranks size their KV cache identically (min over ranks)."""
    dev = torch.device(device)
    if dev.type == "cuda":
        free, total = torch.cuda.mem_get_info(dev)
        n = int((free - reserve_frac * total) // kv_bytes_per_block)
    else:
        n = 512
    if cap is not None:
        n = min(n, cap)
    gloo = group is not None and dist.is_initialized() and dist.get_backend(group) == "gloo"
    t = torch.tensor([n], dtype=torch.int64, device=dev if dev.type == "cuda" and not gloo else "cpu")
    if group is not None and dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return int(t.item())


def worker_loop(model, kv, bcast: StepBroadcaster) -> int:
    """Mirror the driver's forward passes until it broadcasts stop.  Graph
    steps replay this rank's copy of the driver's captured hipGraph (same key,
    same static layout; forward only - sampling is the driver's)."""
    graphs = None

    def graph_buffer(key):
        nonlocal graphs
        if graphs is None:
            from .graphs import GraphRunner
            graphs = GraphRunner(model, kv, 0.0, 0, sample=False)
        return graphs.get(key).buf

    n = 0
    while True:
        msg = bcast.recv(graph_buffer)
        if msg is None:
            return n
        payload, layout = msg
        if isinstance(layout, tuple) and layout[0] == "graph":
            graphs.replay(layout[1])
            model.comm_check()
            n += 1
            continue
        dstep, csrc, cdst = views(payload, layout)
        if csrc.numel():
            ops.copy_blocks(kv.data, csrc, cdst)
        if dstep.token_ids.numel():
            model.forward(dstep, kv)
        model.comm_check()          # K12 peer timeout -> hard failure (lags <= 1 step)
        n += 1
