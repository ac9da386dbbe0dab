"""K13 direct RCCL communicator on the box's single GPU (world size 1: init,
all-reduce / all-gather / reduce-scatter / broadcast are exercised end to end;
multi-rank paths run in the 8-GPU TP bench)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def test_native_rccl_single_rank():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from mcp_amd.parallel.comm import NativeComm
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        c = NativeComm(dist.group.WORLD, "cuda:0")
        x = torch.randn(4096, device="cuda").bfloat16()
        y = x.clone()
        c.all_reduce(y)
        assert torch.equal(x, y)
        g = c.all_gather(x)
        assert g.shape == (1, 4096) and torch.equal(g[0], x)
        f = torch.randn(1024, device="cuda")
        assert torch.equal(c.reduce_scatter(f), f)
        m = f.clone()
        c.all_reduce(m, "max")
        assert torch.equal(m, f)
        c.broadcast(m, 0)
        torch.cuda.synchronize()
        c.close()
        # sequence-parallel pair over the same communicator type: row views
        from mcp_amd.parallel.comm import make_sp_collectives
        rs, ag = make_sp_collectives(dist.group.WORLD, "cuda:0")
        y = torch.randn(6, 64, device="cuda").bfloat16()
        assert rs(y).shape == (6, 64) and torch.equal(rs(y), y)
        assert ag(y[:3]).shape == (3, 64) and torch.equal(ag(y[:3]), y[:3])
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
