"""Split-KV decode attention (K6) microbenchmark: batch-1 / batch-4 decode at
long contexts, the unsplit 1-wave kernel vs the engine's split rule; KV read
bandwidth = K+V bytes of every sequence's context / time.
    python tools/bench_attention_splitkv.py"""
import json
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402
from mcp_amd.engine.batch import StepInputs, choose_kv_splits, pack  # noqa: E402

DEV = "cuda"
Hq, Hkv, D, BS = 32, 8, 128, 64
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def t_us(fn, n=20):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / n * 1e3)
    return round(best, 1)


for ctx in (8192, 32768, 131072):
    for batch in (1, 4):
        nblk = ctx // BS
        nb = nblk * batch
        kc = torch.randn(nb, Hkv, BS, D, device=DEV).bfloat16()
        vc = torch.randn(nb, Hkv, BS, D, device=DEV).bfloat16()
        bt = np.arange(nb, dtype=np.int32).reshape(batch, nblk)
        q = torch.randn(batch, Hq, D, device=DEV).bfloat16()
        step = StepInputs(token_ids=np.zeros(batch, np.int32), positions=np.zeros(batch, np.int32),
                          slots=np.zeros(batch, np.int32), q_start=np.arange(batch, dtype=np.int32),
                          q_len=np.ones(batch, np.int32), ctx_len=np.full(batch, ctx, np.int32),
                          block_table=bt, logit_rows=np.zeros(0, np.int32))
        d = pack(step, Hq // Hkv, DEV)
        r = {"ctx": ctx, "batch": batch}
        ns_rule = choose_kv_splits([1] * batch, [ctx] * batch, Hq // Hkv, Hkv, hq=Hq)
        for ns in sorted({1, 8, 16, 32, 64, 128, ns_rule}):
            d.attn.kv_splits = ns
            us = t_us(lambda: ops.paged_attention(q, kc, vc, d.attn, 1 / math.sqrt(D)))
            r[f"s{ns}_us"] = us
        kv_bytes = 2 * batch * ctx * Hkv * D * 2
        best = min(v for k, v in r.items() if k.endswith("_us"))
        r["rule_splits"] = ns_rule
        r["rule_TBps"] = round(kv_bytes / r[f"s{ns_rule}_us"] / 1e6, 2)
        r["unsplit_TBps"] = round(kv_bytes / r["s1_us"] / 1e6, 2)
        r["best_TBps"] = round(kv_bytes / best / 1e6, 2)
        print(json.dumps(r), flush=True)
        del kc, vc
        torch.cuda.empty_cache()
