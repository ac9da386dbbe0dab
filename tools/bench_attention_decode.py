"""Decode-step attention latency (config 2 / low-QPS config 5 shapes): a few
sequences with 300-4000 keys each and 1-32 new query tokens, Llama-3-8B heads
(32 q / 8 kv, d = 128).  Each case is captured as a hipGraph of REPS attention
calls (as the engine replays them) and timed over replays with HIP events, so
the number is device time per call including the in-graph launch gaps.

    python tools/bench_attention_decode.py [--forms cur,dec] > out.jsonl

``--splits`` = the split counts to try (the engine's choose_kv_splits pick is
always added, key "auto").
"""
import argparse
import json
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mcp_amd.ops as ops  # noqa: E402
from mcp_amd.engine.batch import StepInputs, choose_kv_splits, pack  # noqa: E402

DEV = "cuda"
Hq, Hkv, D, BS = 32, 8, 128, 64
REPS = 20


def time_graph(fn, reps=REPS, rounds=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(rounds):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps * 1e3)
    return round(best, 2)


def case(nseq, ctx, ql, splits, env_forms):
    nblk = (ctx + BS - 1) // BS
    kc = torch.randn(nseq * nblk, Hkv, BS, D, device=DEV).bfloat16()
    vc = torch.randn(nseq * nblk, Hkv, BS, D, device=DEV).bfloat16()
    T = nseq * ql
    q = torch.randn(T, Hq, D, device=DEV).bfloat16()
    out = torch.empty_like(q)
    step = StepInputs(token_ids=np.zeros(T, np.int32), positions=np.zeros(T, np.int32),
                      slots=np.zeros(T, np.int32),
                      q_start=np.arange(nseq, dtype=np.int32) * ql,
                      q_len=np.full(nseq, ql, np.int32), ctx_len=np.full(nseq, ctx, np.int32),
                      block_table=np.arange(nseq * nblk, dtype=np.int32).reshape(nseq, nblk),
                      logit_rows=np.zeros(0, np.int32))
    d = pack(step, Hq // Hkv, DEV)
    auto = choose_kv_splits([ql] * nseq, [ctx] * nseq, Hq // Hkv, Hkv)
    r = {"nseq": nseq, "ctx": ctx, "ql": ql, "auto_splits": auto}
    ref = None
    for form, env in env_forms:
        ops._DECODE_SPLIT = env["MCP_ATTN_DECODE"] == "1"
        # the decode kernel only needs "a split step" (ns > 1); its grid is fixed
        for ns in ([2] if form == "dec" else sorted(set(splits) | {auto})):
            d.attn.kv_splits = ns
            ops.paged_attention(q, kc, vc, d.attn, 1 / math.sqrt(D), out=out)
            torch.cuda.synchronize()
            if ref is None:
                ref = out.float().clone()
            err = float((out.float() - ref).abs().max())
            t = time_graph(lambda: ops.paged_attention(q, kc, vc, d.attn, 1 / math.sqrt(D), out=out))
            r[f"{form}_s{ns}"] = t
            if err > 0.05:
                r[f"{form}_s{ns}_err"] = round(err, 4)
    kv_bytes = nseq * ctx * Hkv * D * 2 * 2
    r["kv_MB"] = round(kv_bytes / 1e6, 2)
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--forms", default="cur")
    ap.add_argument("--splits", default="1,2,4,8,16")
    ap.add_argument("--ctx", default="300,700,1100,2000,4000")
    ap.add_argument("--ql", default="1,4,8,16,32")
    ap.add_argument("--nseq", default="1,2,4")
    a = ap.parse_args()
    forms = {"cur": {"MCP_ATTN_DECODE": "0"}, "dec": {"MCP_ATTN_DECODE": "1"}}
    env_forms = [(f, forms[f]) for f in a.forms.split(",")]
    splits = [int(x) for x in a.splits.split(",")]
    y = torch.zeros(8, device=DEV, dtype=torch.bfloat16)
    print(json.dumps({"empty_kernel_us": time_graph(lambda: ops.add_inplace(y, y))}), flush=True)
    for nseq in [int(x) for x in a.nseq.split(",")]:
        for ctx in [int(x) for x in a.ctx.split(",")]:
            for ql in [int(x) for x in a.ql.split(",")]:
                print(json.dumps(case(nseq, ctx, ql, splits, env_forms)), flush=True)


if __name__ == "__main__":
    main()
