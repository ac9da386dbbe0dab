"""Single-sequence decode attention (config 2 shape: ~700-1100 keys, 1-16
new tokens, Llama-3-8B heads) per split count, fused single launch vs the
per-list launches + combine (ops._MIXED_SPLIT)."""
import json, math, os, sys
import numpy as np, torch
sys.path.insert(0, os.getcwd())
import mcp_amd.ops as ops
from mcp_amd.engine.batch import StepInputs, pack
DEV = "cuda"; Hq, Hkv, D, BS = 32, 8, 128, 64
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
def t_us(fn, n=50):
    fn(); torch.cuda.synchronize(); best = 1e9
    for _ in range(3):
        e0.record()
        for _ in range(n): fn()
        e1.record(); torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / n * 1e3)
    return round(best, 1)
for ctx in (700, 1100):
    for ql in (1, 8, 16):
        nblk = (ctx + BS - 1) // BS
        kc = torch.randn(nblk, Hkv, BS, D, device=DEV).bfloat16()
        vc = torch.randn(nblk, Hkv, BS, D, device=DEV).bfloat16()
        q = torch.randn(ql, Hq, D, device=DEV).bfloat16()
        step = StepInputs(token_ids=np.zeros(ql, np.int32), positions=np.zeros(ql, np.int32),
                          slots=np.zeros(ql, np.int32), q_start=np.zeros(1, np.int32),
                          q_len=np.full(1, ql, np.int32), ctx_len=np.full(1, ctx, np.int32),
                          block_table=np.arange(nblk, dtype=np.int32)[None], logit_rows=np.zeros(0, np.int32))
        d = pack(step, Hq // Hkv, DEV)
        r = {"ctx": ctx, "ql": ql}
        for mixed in (True, False):
            ops._MIXED_SPLIT = mixed
            for ns in (1, 2, 4, 8, 16):
                if ns == 1 and not mixed: continue
                d.attn.kv_splits = ns
                r[f"{'m' if mixed else 'l'}{ns}"] = t_us(lambda: ops.paged_attention(q, kc, vc, d.attn, 1 / math.sqrt(D)))
        print(json.dumps(r), flush=True)
