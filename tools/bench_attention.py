"""Attention microbenchmark at the headline bench's shapes: a 4096-token step
of 256 requests (16 new tokens each) sharing a 704-token registry prefix, each
with ~200 keys of its own; Llama-3-8B heads (32 q / 8 kv, d=128).  Times the
shared-prefix pass and the per-request pass separately (torch events)."""
import json
import math
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import mcp_amd  # noqa: E402,F401
from mcp_amd import ops  # noqa: E402
from mcp_amd.engine.batch import StepInputs, pack  # noqa: E402

dev = "cuda"
Hq, Hkv, D = 32, 8, 128
# argv[1]: new tokens per request (16: 4-wave items; <= 8: 1-wave decode items)
# "a:b" alternates requests of a and b new tokens (mixed decode / jump-forward steps)
qls = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "16").split(":")]
import os
S, prefix = int(os.environ.get("ATTN_S", "256")), int(os.environ.get("ATTN_PREFIX", "704"))  # ATTN_S: requests in the step
ql_s = np.array([qls[s % len(qls)] for s in range(S)], np.int32)
ql = int(ql_s.max())
own = int(os.environ.get("ATTN_OWN", "200"))
nb_pre = prefix // 64
rng = np.random.default_rng(0)
blocks_per_seq = (prefix + own + ql + 63) // 64
nb = nb_pre + S * (blocks_per_seq - nb_pre) + 8
kc = torch.randn(nb, Hkv, 64, D, device=dev).bfloat16()
vc = torch.randn(nb, Hkv, 64, D, device=dev).bfloat16()
T = int(ql_s.sum())
q = torch.randn(T, Hq, D, device=dev).bfloat16()
bt = np.zeros((S, blocks_per_seq), np.int32)
nxt = nb_pre
for s in range(S):
    bt[s, :nb_pre] = np.arange(nb_pre)
    for j in range(nb_pre, blocks_per_seq):
        bt[s, j] = nxt
        nxt += 1
ctx = (prefix + own + ql_s).astype(np.int32)
qs = np.concatenate([[0], np.cumsum(ql_s)[:-1]]).astype(np.int32)
step = StepInputs(token_ids=np.zeros(T, np.int32), positions=np.zeros(T, np.int32),
                  slots=np.full(T, -1, np.int32), q_start=qs, q_len=ql_s,
                  ctx_len=ctx, block_table=bt, logit_rows=np.zeros(0, np.int32),
                  kv_begin=np.full(S, prefix, np.int32), pre_bt=np.arange(nb_pre, dtype=np.int32),
                  pre_tokens=T)
d = pack(step, Hq // Hkv, dev)
d.attn.own_tiles = int(-(-(own + ql) // 64))      # as the engine's layout carries it
scale = 1 / math.sqrt(D)
L = ops.lib()
pre_o = torch.empty_like(q)
pre_lse = torch.empty(T, Hq, device=dev)
out = torch.empty_like(q)


def t_prefix():
    L.prefix_attention(q, kc, vc, pre_o, pre_lse, d.attn.pre_bt, d.attn.pre_keys, d.attn.pre_tokens, scale)


def t_own():
    for nw, ws, wq in d.attn.work_lists():
        L.paged_attention(q, kc, vc, out, d.attn.q_start, d.attn.q_len, d.attn.ctx_len,
                          d.attn.block_table, ws, wq, nw, scale, kv_begin=d.attn.kv_begin,
                          pre_o=pre_o, pre_lse=pre_lse)


def t_full():          # the production entry point (prefix pass + work lists)
    ops.paged_attention(q, kc, vc, d.attn, scale, out=out)


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


tp, to, tf = timeit(t_prefix), timeit(t_own), timeit(t_full)
fl_pre = 4.0 * T * Hq * prefix * D
fl_own = 4.0 * T * Hq * (own + ql / 2) * D
# correctness of the cascade against the plain per-request pass over all keys
ref = torch.empty_like(q)
for nw, ws, wq in d.attn.work_lists():
    L.paged_attention(q, kc, vc, ref, d.attn.q_start, d.attn.q_len, d.attn.ctx_len,
                      d.attn.block_table, ws, wq, nw, scale)
t_prefix()
t_own()
err = ((out.float() - ref.float()).norm() / ref.norm()).item()
print(json.dumps({"S": S, "own": own, "ql": sys.argv[1] if len(sys.argv) > 1 else "16", "full_us": round(tf, 1), "prefix_us": round(tp, 1), "prefix_tflops": round(fl_pre / tp / 1e6, 1),
                  "own_us": round(to, 1), "own_tflops": round(fl_own / to / 1e6, 1),
                  "cascade_vs_plain_rel_err": err}))
