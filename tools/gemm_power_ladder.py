"""Energy / issue ladder of the headline GEMM.

Round 5 inferred "power limit" from MFMA busy x clock staying at ~1.18 G/s
across two kernel versions.  This measures it: the production 256-row AGPR
kernel (csrc/gemm256d.hip) and three probe forms of the same launch
(``PROBE``: 1 = the MFMA issue alone, 2 = + the ds_read fragment schedule and
barriers, 3 = + the LDS-DMA; 0 = production, i.e. + the epilogue stores),
each timed and then run back to back for a few seconds while a side thread
samples the board (amdsmi: socket power, GFX clock).  Per rung: us, TFLOP/s,
mean W, mean MHz, pJ per FLOP.

    python tools/gemm_power_ladder.py                 # all rungs, both shapes, JSON lines
    python tools/gemm_power_ladder.py --rung 2 --shape gu --iters 20   # one rung (rocprofv3 --pmc passes)

Shapes: gu = gate|up + SwiGLU, M = 2560 x N = 28672 x K = 4096 (the headline's
largest GEMM, epilogue 2); down = M 2560 x N 4096 x K 14336, plain epilogue.
Weights rotate over 2 copies (> the 256 MB Infinity Cache for gu), as in
serving.  Synthetic data (randn), timing only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mcp_amd.ops as ops  # noqa: E402

SHAPES = {"gu": (2560, 28672, 4096, 2), "down": (2560, 4096, 14336, 0)}
RUNGS = {1: "MFMA issue only", 2: "+ ds_read fragments + barriers", 3: "+ LDS-DMA (mainloop)",
         0: "production (+ epilogue stores)"}


class Sampler:
    """Socket power (W) and GFX clock (MHz) every ``period`` s via amdsmi."""

    def __init__(self, period: float = 0.02):
        self.period = period
        self.ok = False
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            self.smi = amdsmi
            self.h = amdsmi.amdsmi_get_processor_handles()[0]
            self.ok = True
        except Exception as e:  # noqa: BLE001
            self.err = repr(e)

    def read(self):
        smi = self.smi
        p = smi.amdsmi_get_power_info(self.h)
        w = p.get("current_socket_power")
        if not isinstance(w, (int, float)) or w <= 0:
            w = p.get("average_socket_power")
        c = smi.amdsmi_get_clock_info(self.h, smi.AmdSmiClkType.GFX)
        return float(w), float(c.get("clk", 0))

    def run(self, fn, seconds: float):
        """Call ``fn`` repeatedly for ``seconds`` while sampling; mean W and MHz."""
        samples = []
        stop = threading.Event()

        def poll():
            while not stop.is_set():
                try:
                    samples.append(self.read())
                except Exception:  # noqa: BLE001
                    pass
                time.sleep(self.period)
        th = threading.Thread(target=poll, daemon=True)
        t0 = time.perf_counter()
        th.start()
        n = 0
        while time.perf_counter() - t0 < seconds:
            for _ in range(8):
                fn(n)
                n += 1
            torch.cuda.synchronize()
        stop.set()
        th.join()
        # drop the first quarter (clock / power settling)
        s = samples[len(samples) // 4:] or samples
        if not s:
            return None, None
        return sum(x[0] for x in s) / len(s), sum(x[1] for x in s) / len(s)


def bench(shape: str, rungs, iters: int, power_s: float, sampler):
    M, N, K, epi = SHAPES[shape]
    L = ops.lib()
    X = torch.randn(M, K, device="cuda").bfloat16()
    Ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(2)]
    Y = torch.empty(M, N // 2 if epi == 2 else N, device="cuda", dtype=torch.bfloat16)
    flop = 2.0 * M * N * K
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = []
    for r in rungs:
        def fn(i, r=r):
            L.gemm_probe(X, Ws[i & 1], Y, epi, r)
        for i in range(4):
            fn(i)
        torch.cuda.synchronize()
        e0.record()
        for i in range(iters):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / iters * 1e3
        rec = {"shape": shape, "M": M, "N": N, "K": K, "rung": r, "form": RUNGS[r],
               "us": round(us, 1), "tflops": round(flop / us / 1e6, 1)}
        if sampler is not None and sampler.ok and power_s > 0:
            w, mhz = sampler.run(fn, power_s)
            if w is not None:
                rec.update(watts=round(w, 1), gfx_mhz=round(mhz),
                           pj_per_flop=round(w * us * 1e-6 / flop * 1e12, 4))
        print(json.dumps(rec), flush=True)
        out.append(rec)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", choices=list(SHAPES) + ["all"], default="all")
    ap.add_argument("--rung", type=int, default=-1, help="one rung (0-3); default all")
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--power-s", type=float, default=4.0, help="seconds of sampling per rung (0: off)")
    a = ap.parse_args()
    rungs = [a.rung] if a.rung >= 0 else [1, 2, 3, 0]
    sampler = Sampler() if a.power_s > 0 else None
    if sampler is not None and not sampler.ok:
        print(json.dumps({"power": "unavailable", "error": sampler.err}), flush=True)
    for shape in (list(SHAPES) if a.shape == "all" else [a.shape]):
        bench(shape, rungs, a.iters, a.power_s, sampler)


if __name__ == "__main__":
    main()
