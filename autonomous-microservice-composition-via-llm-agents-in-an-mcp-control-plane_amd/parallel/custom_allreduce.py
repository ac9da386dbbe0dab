"""K12 custom all-reduce over xGMI peer-to-peer.

Tensor-parallel decode all-reduces are small ([B, 8192] bf16 per row-parallel
projection, 2 per layer, C1/C2) and RCCL's ring pays 2(N-1) latency-bound
hops for each of them.  ``csrc/custom_allreduce.hip`` instead reads every
peer's IPC-mapped staging buffer directly over the point-to-point xGMI links:

* one-shot for small messages (one barrier, sum of N buffers per rank);
* two-shot (reduce-scatter + all-gather through the buffers, two barriers)
  for mid-size messages;
* anything larger than the staging buffer falls back to RCCL (``eligible``).

Set-up exchanges the ``hipIpcMemHandle_t`` of each rank's staging buffer and
signal array over the process group (gloo or RCCL), then opens the peers'
handles.  The reference has no collectives at all.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .. import ops

# one-shot / two-shot crossover: MCP_CAR_ONE_SHOT_MAX, else the xGMI cost
# model's at this world size (parallel/xgmi_model.py: ~307 KB at 8 ranks)
_ONE_SHOT_ENV = os.environ.get("MCP_CAR_ONE_SHOT_MAX")
# workgroups per call (0: one per 4 x 512 16-B vectors, at most 128).  Every
# rank's blocks spin on flags the peers' blocks raise, so all ranks' blocks
# must be resident at once: on a node each rank has its own GPU, but ranks
# sharing one device (the 8-process tests) must cap it (MCP_CAR_BLOCKS=16)
MAX_BLOCKS = int(os.environ.get("MCP_CAR_BLOCKS", "0"))


class CustomAllReduce:
    def __init__(self, group, device, max_bytes: int = 8 << 20):
        self.group = group
        self.device = torch.device(device)
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.max_bytes = max_bytes
        from .xgmi_model import one_shot_max_bytes
        self.one_shot_max = int(_ONE_SHOT_ENV) if _ONE_SHOT_ENV else one_shot_max_bytes(self.world)
        lib = ops.lib()
        self._lib = lib
        hb = lib.car_handle_bytes()
        mine = torch.zeros(hb, dtype=torch.uint8)
        with torch.cuda.device(self.device):
            self._h = lib.car_init(self.rank, self.world, max_bytes, mine)
        gathered = [None] * self.world
        dist.all_gather_object(gathered, bytes(mine.numpy().tobytes()), group=group)
        allh = torch.frombuffer(bytearray(b"".join(gathered)), dtype=torch.uint8).clone()
        with torch.cuda.device(self.device):
            lib.car_connect(self._h, allh)
        dist.barrier(group=group)

    def eligible(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous()
                and t.numel() % 8 == 0 and 0 < t.numel() * 2 <= self.max_bytes)

    @staticmethod
    def ss_eligible(t: torch.Tensor) -> bool:
        """Rows the kernel can add the fused-norm statistic of (H >= 512, % 8)."""
        h = t.shape[-1]
        return h % 8 == 0 and h >= 512

    def __call__(self, t: torch.Tensor, out: torch.Tensor = None, mode: int = 0,
                 blocks: int = 0, ss_out: torch.Tensor = None) -> torch.Tensor:
        """Sum ``t`` over the group (in place unless ``out`` is given).
        mode: 0 auto, 1 one-shot, 2 two-shot.  ``ss_out`` (int64, zeroed):
        also add every summed row's fixed-point sum of squares (the next
        layer's fused RMSNorm statistic; ``ss_eligible`` rows)."""
        out = t if out is None else out
        if mode == 0:
            mode = 1 if t.numel() * 2 <= self.one_shot_max else 2
        self._lib.car_run(self._h, t, out, mode, blocks or MAX_BLOCKS, ss_out)
        return out

    def check(self) -> None:
        """Raise if any barrier of a previous call timed out waiting for a peer."""
        if self._lib.car_error(self._h):
            raise RuntimeError("custom all-reduce: a peer did not arrive (barrier timeout)")

    def close(self) -> None:
        if self._h:
            self._lib.car_destroy(self._h)
            self._h = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
