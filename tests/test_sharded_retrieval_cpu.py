"""C6: corpus-sharded top-k over 2 gloo ranks equals single-rank top-k."""
import os
import socket

import torch
import torch.multiprocessing as mp


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import mcp_amd  # noqa: F401
    from mcp_amd.retrieval.sharded import ShardedIndex
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(0)
    corpus = torch.nn.functional.normalize(torch.randn(1001, 64, generator=g), dim=-1)
    queries = torch.nn.functional.normalize(torch.randn(5, 64, generator=g), dim=-1)
    idx = ShardedIndex(dist.group.WORLD, "cpu")
    idx.set_corpus(corpus)
    v, i = idx.search(queries, 7)
    # plain lists: a torch tensor in the queue is shared by file descriptor,
    # which the parent can no longer fetch once this process has exited
    q.put((rank, v.tolist(), i.tolist()))
    dist.destroy_process_group()


def test_sharded_topk_matches_global():
    from mcp_amd.retrieval.sharded import ShardedIndex, shard_range
    assert [shard_range(10, r, 3) for r in range(3)] == [(0, 4), (4, 7), (7, 10)]
    g = torch.Generator().manual_seed(0)
    corpus = torch.nn.functional.normalize(torch.randn(1001, 64, generator=g), dim=-1)
    queries = torch.nn.functional.normalize(torch.randn(5, 64, generator=g), dim=-1)
    ref = ShardedIndex(None, "cpu")
    ref.set_corpus(corpus)
    rv, ri = ref.search(queries, 7)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=30)
    for rank, v, i in out:
        assert torch.allclose(torch.tensor(v), rv, atol=1e-6)
        assert torch.equal(torch.tensor(i, dtype=ri.dtype), ri)
