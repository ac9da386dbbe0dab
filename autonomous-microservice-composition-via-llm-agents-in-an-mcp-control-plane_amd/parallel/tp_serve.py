"""Tensor-parallel planner behind the API (``MCP_TP=t``; SURVEY §2.3 "Megatron
1-D TP", BASELINE config 4: Llama-3-70B at TP=8 over xGMI).

The reference serves ``/plan`` from one process that calls a remote LLM
(control_plane.py:137,140-142,69-73).  With ``MCP_TP=t`` the API process
becomes TP rank 0, the *driver*: it owns the FastAPI app, the scheduler
thread, the block allocator, the grammar state and sampling
(``LocalPlanner`` + ``LLMEngine(bcast=...)``).  Ranks 1..t-1 are fresh worker
processes (spawned before this process touches the GPU, one per device) that
rebuild the same sharded model and mirror every forward from the step
descriptors the driver broadcasts (``engine.tp.worker_loop``).  The
row-parallel projections all-reduce through ``parallel.comm.AllReduce``:
K12 over xGMI for decode-sized messages, RCCL above.

Devices: ``MCP_TP_DEVICES`` (comma list, default ``cuda:0..t-1``, or ``cpu``
when no GPU is visible); process-group backend ``MCP_TP_BACKEND`` (default
``nccl`` on GPUs, ``gloo`` on CPU).  Several ranks may share one GPU for
tests (gloo group, every all-reduce through K12: ``MCP_COMM=torch``,
``MCP_CAR_MAX_BYTES`` large).
"""
from __future__ import annotations

import multiprocessing as mp
import os
from typing import List, Optional

import torch
import torch.distributed as dist

from ..planner.local import LocalPlanner
from ..planner.tokenizer import tokenizer_for


def _default_devices(tp: int) -> List[str]:
    env = os.environ.get("MCP_TP_DEVICES")
    if env:
        devs = [d.strip() for d in env.split(",") if d.strip()]
        if len(devs) != tp:
            raise ValueError(f"MCP_TP_DEVICES lists {len(devs)} devices for MCP_TP={tp}")
        return devs
    if torch.cuda.device_count() > 0:       # counts devices without initialising HIP
        if torch.cuda.device_count() < tp:
            raise RuntimeError(f"MCP_TP={tp} needs {tp} GPUs, found {torch.cuda.device_count()}")
        return [f"cuda:{i}" for i in range(tp)]
    return ["cpu"] * tp


def build_rank(model_name: str, rank: int, world: int, device: str, seed: int,
               kv_blocks: Optional[int], full_weights_seed: Optional[int] = None):
    """Sharded model + agreed KV block count + step broadcaster of one rank
    (the process group is already initialised).  ``full_weights_seed``: shard
    one full random init (tests compare against the TP=1 model of the same
    weights) instead of drawing each shard independently."""
    from ..engine.kv_cache import KVCache
    from ..engine.tp import agree_num_blocks
    from ..models.llama import (LlamaModel, LlamaWeights, get_config, random_weights,
                                shard_layer)
    from .comm import StepBroadcaster
    group = dist.group.WORLD
    if os.path.isdir(model_name):            # an HF checkpoint: this rank's shards only
        from ..models.weights import model_from_checkpoint
        model = model_from_checkpoint(model_name, device, tp_rank=rank, tp=world, tp_group=group)
        cfg = model.cfg
    elif full_weights_seed is None:
        cfg = get_config(model_name)
        model = LlamaModel.random(model_name, device, seed=seed, tp_rank=rank, tp=world,
                                  tp_group=group)
    else:
        cfg = get_config(model_name)
        full = random_weights(cfg, device, seed=full_weights_seed)
        sh = LlamaWeights(embed=full.embed, final_norm=full.final_norm, lm_head=full.lm_head,
                          layers=[shard_layer(l, cfg, rank, world) for l in full.layers])
        del full
        model = LlamaModel(cfg, sh, device, tp_rank=rank, tp=world, tp_group=group)
    per_block = KVCache.bytes_per_block(cfg.layers, model.hkv, cfg.head_dim)
    nb = agree_num_blocks(per_block, device, group, cap=kv_blocks or (None if str(device).startswith("cuda") else 512))
    return model, nb, StepBroadcaster(group, device)


def _worker_main(rank: int, world: int, port: int, device: str, backend: str, model_name: str,
                 seed: int, kv_blocks: Optional[int], env: dict,
                 full_weights_seed: Optional[int] = None) -> None:
    os.environ.update(env)
    from ..engine.kv_cache import KVCache
    from ..engine.tp import worker_loop
    if device.startswith("cuda"):
        torch.cuda.set_device(torch.device(device))
    kw = {"device_id": torch.device(device)} if backend == "nccl" else {}
    dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world, **kw)
    model, nb, bc = build_rank(model_name, rank, world, device, seed, kv_blocks, full_weights_seed)
    kv = KVCache(model.cfg.layers, model.hkv, model.cfg.head_dim, nb, device)
    worker_loop(model, kv, bc)
    dist.destroy_process_group()


class TPPlanner(LocalPlanner):
    """``LocalPlanner`` on a TP driver; ``launch`` starts the worker ranks."""

    _workers: List = []

    @classmethod
    def launch(cls, settings, registry, devices: Optional[List[str]] = None,
               backend: Optional[str] = None, full_weights_seed: Optional[int] = None,
               temperature: Optional[float] = None) -> "TPPlanner":
        from ..engine.engine import LLMEngine
        from ..retrieval.store import SchemaIndex
        from .launch import free_port
        tp = int(settings.tp)
        devices = devices or _default_devices(tp)
        backend = backend or os.environ.get("MCP_TP_BACKEND") or \
            ("nccl" if devices[0].startswith("cuda") else "gloo")
        port = free_port()
        ctx = mp.get_context("spawn")
        env = {k: v for k, v in os.environ.items() if k.startswith("MCP_") or k.startswith("HSA_")}
        kvb = settings.kv_blocks or None
        workers = []
        for r in range(1, tp):              # fresh processes: spawned before any GPU call here
            p = ctx.Process(target=_worker_main, daemon=True,
                            args=(r, tp, port, devices[r], backend, settings.model, settings.seed,
                                  kvb, env, full_weights_seed))
            p.start()
            workers.append(p)
        dev = devices[0]
        if dev.startswith("cuda"):
            torch.cuda.set_device(torch.device(dev))
        kw = {"device_id": torch.device(dev)} if backend == "nccl" else {}
        dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=0,
                                world_size=tp, **kw)
        model, nb, bc = build_rank(settings.model, 0, tp, dev, settings.seed, kvb, full_weights_seed)
        eng = LLMEngine(model, num_blocks=nb, max_batch=settings.max_batch,
                        max_step_tokens=settings.max_step_tokens,
                        temperature=settings.temperature if temperature is None else temperature,
                        seed=settings.seed, bcast=bc)
        retr = SchemaIndex(registry, dim=settings.embed_dim, device=dev)
        retr.refresh()
        retr.start_background()
        planner = cls(eng, registry, tokenizer=tokenizer_for(settings.model),
                      max_nodes=settings.max_nodes, retriever=retr,
                      retrieval_threshold=settings.retrieval_threshold, topk=settings.topk)
        planner._workers = workers
        return planner

    def shutdown(self) -> None:
        """Stop the scheduler thread, release the workers, tear the group down."""
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=30)
        if not self._workers:
            return
        try:
            self.engine.shutdown_workers()
        finally:
            for p in self._workers:
                p.join(timeout=60)
                if p.is_alive():
                    p.kill()
            self._workers = []
            if dist.is_initialized():
                dist.destroy_process_group()

    async def aclose(self):
        self.shutdown()
