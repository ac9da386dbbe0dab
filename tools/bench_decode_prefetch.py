"""Decode-layer chain with and without Infinity-Cache weight prefetch on a side
stream (config 2 / 5 shapes: Llama-3-8B TP=1, M = 1-32 tokens).

One "layer" = QKV GEMM, paged attention over CTX keys, o + residual, SwiGLU
gate|up, down + residual - the weight-streaming decode step of
models.llama.  NL layers of distinct random weights (more bytes than the
256 MiB Infinity Cache, so nothing stays resident between passes) run back to
back; ms per layer is reported:

* ``base``: everything on the main stream;
* ``pf``:   while GEMM g runs (and the attention before o), a side stream reads
  the weights of the NEXT GEMM (``ops.lib().prefetch``), fork / join by events;
* ``*_g``:  the same captured in one hipGraph.

    python tools/bench_decode_prefetch.py --m 1,4,16 > out.jsonl
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
H, F, Hq, Hkv, D, BS = 4096, 14336, 32, 8, 128, 64


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="1,4,16")
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--ctx", type=int, default=1000)
    ap.add_argument("--blocks", default="256")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    L = lib = ops.lib()
    g = torch.Generator(device=DEV).manual_seed(0)

    def rnd(*s):
        return (torch.randn(*s, device=DEV, generator=g) * 0.02).bfloat16()

    Ws = [dict(qkv=rnd((Hq + 2 * Hkv) * D, H), o=rnd(H, Hq * D), gu=rnd(2 * F, H), down=rnd(H, F))
          for _ in range(a.layers)]
    nblk = (a.ctx + BS - 1) // BS
    kc = rnd(nblk, Hkv, BS, D)
    vc = rnd(nblk, Hkv, BS, D)
    sink = torch.zeros(16, dtype=torch.int32, device=DEV)
    side = torch.cuda.Stream()
    for blocks in [int(b) for b in a.blocks.split(",")]:
        for M in [int(x) for x in a.m.split(",")]:
            x = rnd(M, H)
            q = rnd(M, Hq, D)
            qkv = torch.empty(M, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
            att = torch.empty(M, Hq, D, device=DEV, dtype=torch.bfloat16)
            act = torch.empty(M, F, device=DEV, dtype=torch.bfloat16)
            step = StepInputs(token_ids=np.zeros(M, np.int32), positions=np.zeros(M, np.int32),
                              slots=np.zeros(M, np.int32), q_start=np.zeros(1, np.int32),
                              q_len=np.full(1, M, np.int32), ctx_len=np.full(1, a.ctx, np.int32),
                              block_table=np.arange(nblk, dtype=np.int32)[None],
                              logit_rows=np.zeros(0, np.int32))
            d = pack(step, Hq // Hkv, DEV)
            d.attn.kv_splits = choose_kv_splits([M], [a.ctx], Hq // Hkv, Hkv)
            scale = 1 / math.sqrt(D)

            def pf(w):
                lib.prefetch(w, 0, w.numel() * 2, blocks, sink)

            def run(prefetch):
                main = torch.cuda.current_stream()
                for li, w in enumerate(Ws):
                    nxt = Ws[(li + 1) % len(Ws)]
                    seq = [("qkv", w["o"]), ("attn", w["gu"]), ("o", None), ("gu", w["down"]),
                           ("down", nxt["qkv"])]
                    for name, target in seq:
                        if prefetch and target is not None:
                            side.wait_stream(main)
                            with torch.cuda.stream(side):
                                pf(target)
                        if name == "qkv":
                            ops.gemm(x, w["qkv"], out=qkv)
                        elif name == "attn":
                            ops.paged_attention(q, kc, vc, d.attn, scale, out=att)
                        elif name == "o":
                            ops.gemm(att.view(M, Hq * D), w["o"], R=x, out=x)
                        elif name == "gu":
                            ops.gemm_silu(x, w["gu"], out=act)
                        else:
                            ops.gemm(act, w["down"], R=x, out=x)
                if prefetch:
                    main.wait_stream(side)

            def timed(fn):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                fn()
                torch.cuda.synchronize()
                best = 1e9
                for _ in range(a.reps):
                    e0.record()
                    fn()
                    e1.record()
                    torch.cuda.synchronize()
                    best = min(best, e0.elapsed_time(e1))
                return round(best / len(Ws) * 1e3, 1)          # us per layer

            def graphed(prefetch):
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    run(prefetch)
                torch.cuda.current_stream().wait_stream(s)
                torch.cuda.synchronize()
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr):
                    run(prefetch)
                return gr.replay

            r = {"M": M, "ctx": a.ctx, "layers": a.layers, "blocks": blocks,
                 "kv_splits": d.attn.kv_splits,
                 "floor_us": round((Ws[0]["qkv"].numel() + Ws[0]["o"].numel() + Ws[0]["gu"].numel()
                                    + Ws[0]["down"].numel()) * 2 / 6.3e6, 1)}
            r["base"] = timed(lambda: run(False))
            r["pf"] = timed(lambda: run(True))
            r["base_g"] = timed(graphed(False))
            r["pf_g"] = timed(graphed(True))
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
