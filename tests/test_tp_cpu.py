"""Tensor parallelism on CPU with gloo, world_size 2.

* the Megatron-sharded forward (column-parallel Wqkv / Wgate|up, row-parallel
  Wo / Wdown + all-reduce) equals the unsharded forward;
* the sequence-parallel forward (reduce-scatter -> fused add+RMSNorm on T/tp
  rows -> all-gather, ``MCP_SEQ_PARALLEL``) equals it too, also for a token
  count that tp does not divide (padded rows);
* the driver/worker engine (rank 0 schedules, samples and broadcasts step
  descriptors, rank 1 mirrors the forward) plans valid DAGs and shuts down.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _step_inputs(q_lens=(70, 5, 1)):
    from mcp_amd.engine.batch import StepInputs
    q_lens, ctx = list(q_lens), list(q_lens)
    T = sum(q_lens)
    rng = np.random.RandomState(0)
    ids = rng.randint(0, 2000, T).astype(np.int32)
    pos = np.concatenate([np.arange(c - q, c) for q, c in zip(q_lens, ctx)]).astype(np.int32)
    blocks = [[0, 1], [2], [3]]
    bt = np.zeros((3, 2), np.int32)
    for i, b in enumerate(blocks):
        bt[i, :len(b)] = b
    slots = np.concatenate([np.asarray(blocks[i])[p // 64] * 64 + p % 64
                            for i, p in enumerate(np.split(pos, np.cumsum(q_lens)[:-1]))]).astype(np.int32)
    return StepInputs(token_ids=ids, positions=pos, slots=slots,
                      q_start=np.concatenate([[0], np.cumsum(q_lens)[:-1]]).astype(np.int32),
                      q_len=np.array(q_lens, np.int32),
                      ctx_len=np.array(ctx, np.int32), block_table=bt,
                      logit_rows=(np.cumsum(q_lens) - 1).astype(np.int32))


def _forward_worker(rank, world, port, out_dir, sp=False, q_lens=(70, 5, 1)):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    from mcp_amd.engine.batch import pack
    from mcp_amd.engine.kv_cache import KVCache
    from mcp_amd.models.llama import LlamaModel, LlamaWeights, get_config, random_weights, shard_layer
    cfg = get_config("tiny-tp")
    full = random_weights(cfg, "cpu", seed=3)
    step = pack(_step_inputs(q_lens), cfg.group, "cpu")
    ref_model = LlamaModel(cfg, full, "cpu")
    kv1 = KVCache(cfg.layers, cfg.kv_heads, cfg.head_dim, 8, "cpu")
    h_ref = ref_model.forward(step, kv1).float()
    sh = LlamaWeights(embed=full.embed, final_norm=full.final_norm, lm_head=full.lm_head,
                      layers=[shard_layer(l, cfg, rank, world) for l in full.layers])
    model = LlamaModel(cfg, sh, "cpu", tp_rank=rank, tp=world, tp_group=dist.group.WORLD,
                       seq_parallel=sp)
    assert model.seq_parallel == sp
    kv = KVCache(cfg.layers, cfg.kv_heads // world, cfg.head_dim, 8, "cpu")
    h = model.forward(step, kv).float()
    err = ((h - h_ref).norm() / h_ref.norm()).item()
    with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
        f.write(str(err))
    dist.destroy_process_group()


def _engine_worker(rank, world, port, out_dir, sp=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MCP_SEQ_PARALLEL=str(int(sp)))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    import json
    from mcp_amd.engine.engine import LLMEngine
    from mcp_amd.engine.kv_cache import KVCache
    from mcp_amd.engine.tp import agree_num_blocks, worker_loop
    from mcp_amd.models.llama import LlamaModel
    from mcp_amd.parallel.comm import StepBroadcaster
    from mcp_amd.planner.local import LocalPlanner
    from mcp_amd.planner.prompt import synthetic_intent
    from mcp_amd.registry import MemoryRegistry, synthetic_registry
    model = LlamaModel.random("tiny-tp", "cpu", seed=2, tp_rank=rank, tp=world, tp_group=dist.group.WORLD)
    nb = agree_num_blocks(1, "cpu", dist.group.WORLD, cap=256)
    bc = StepBroadcaster(dist.group.WORLD, "cpu", src=0)
    if rank == 0:
        eng = LLMEngine(model, num_blocks=nb, max_batch=8, max_step_tokens=2048, bcast=bc)
        reg = MemoryRegistry(synthetic_registry(5, seed=9))
        planner = LocalPlanner(eng, reg, max_nodes=3)
        dags = planner.plan_many([synthetic_intent(i) for i in range(3)])
        eng.shutdown_workers()
        with open(os.path.join(out_dir, "dags.json"), "w") as f:
            json.dump({"dags": dags, "names": [s.name for s in reg.list_services()],
                       "free": eng.alloc.num_free, "nb": nb}, f)
    else:
        kv = KVCache(model.cfg.layers, model.hkv, model.cfg.head_dim, nb, "cpu")
        n = worker_loop(model, kv, bc)
        with open(os.path.join(out_dir, "worker.txt"), "w") as f:
            f.write(str(n))
    dist.destroy_process_group()


def test_tp2_forward_matches_tp1(tmp_path):
    mp.spawn(_forward_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        err = float(open(tmp_path / f"r{r}.txt").read())
        assert err < 2e-2, err


@pytest.mark.parametrize("q_lens", [(70, 5, 1), (70, 4, 1)])
def test_tp2_sequence_parallel_forward_matches_tp1(tmp_path, q_lens):
    mp.spawn(_forward_worker, args=(2, _free_port(), str(tmp_path), True, q_lens), nprocs=2,
             join=True)
    for r in range(2):
        err = float(open(tmp_path / f"r{r}.txt").read())
        assert err < 2e-2, err


@pytest.mark.parametrize("sp", [False, True])
def test_tp2_driver_worker_engine(tmp_path, sp):
    import json
    from mcp_amd.orchestrator import validate_dag
    mp.spawn(_engine_worker, args=(2, _free_port(), str(tmp_path), sp), nprocs=2, join=True)
    out = json.load(open(tmp_path / "dags.json"))
    for d in out["dags"]:
        validate_dag(d, out["names"])
    assert out["free"] == out["nb"]
    assert int(open(tmp_path / "worker.txt").read()) > 0
