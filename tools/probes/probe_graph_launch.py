"""Does a hipGraph replay return before the GPU has run it?

Config 2's trace puts ~3.7 ms of host time inside ``engine.launch`` per
decision step - about one whole forward - so the host cannot be ahead of the
GPU.  This times ``CUDAGraph.replay()`` (host return) against the graph's GPU
time, for graphs of N kernels of ~T us each, and a plain eager launch of the
same kernels.  One JSON line per case.
"""
import json
import time

import torch


def main():
    dev = torch.device("cuda")
    x = torch.zeros(4 << 20, device=dev)             # 16 MB: a few us per pass
    for n in (32, 128, 320):
        def body():
            for _ in range(n):
                x.add_(1.0)
        body()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            body()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        rows = []
        for _ in range(10):
            t0 = time.perf_counter()
            g.replay()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            rows.append((t1 - t0, t2 - t0))
        rows.sort(key=lambda r: r[1])
        h, tot = rows[len(rows) // 2]
        # back to back: the second replay's host return
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        t1 = time.perf_counter()
        g.replay()
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        # eager
        t4 = time.perf_counter()
        body()
        t5 = time.perf_counter()
        torch.cuda.synchronize()
        t6 = time.perf_counter()
        print(json.dumps({"kernels": n, "replay_host_us": round(h * 1e6, 1),
                          "replay_total_us": round(tot * 1e6, 1),
                          "b2b_first_host_us": round((t1 - t0) * 1e6, 1),
                          "b2b_second_host_us": round((t2 - t1) * 1e6, 1),
                          "b2b_total_us": round((t3 - t0) * 1e6, 1),
                          "eager_host_us": round((t5 - t4) * 1e6, 1),
                          "eager_total_us": round((t6 - t4) * 1e6, 1)}), flush=True)


def ours():
    """The same for graphs of this repo's kernels (skinny / stream GEMMs at
    decode M, with and without the residual + statistic epilogue)."""
    import mcp_amd.ops as ops
    dev = torch.device("cuda")
    X = torch.randn(16, 4096, device=dev, dtype=torch.bfloat16)
    W = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16) * 0.02
    Wg = torch.randn(2 * 14336, 4096, device=dev, dtype=torch.bfloat16) * 0.02
    R = torch.randn(16, 4096, device=dev, dtype=torch.bfloat16)
    ss = torch.zeros(16, dtype=torch.int64, device=dev)
    Y = torch.empty(16, 4096, device=dev, dtype=torch.bfloat16)
    H = torch.empty(16, 14336, device=dev, dtype=torch.bfloat16)
    x = torch.zeros(4 << 20, device=dev)
    cases = {
        "gemm": lambda: ops.gemm(X, W, out=Y),
        "gemm_res_ss": lambda: ops.gemm(X, W, R=R, out=Y, ss_out=ss),
        "gemm_silu": lambda: ops.gemm_silu(X, Wg, out=H),
        "torch_add": lambda: x.add_(1.0),
    }
    for name, f in cases.items():
        for n in (64, 192):
            def body():
                for _ in range(n):
                    f()
            body()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                body()
            g.replay()
            torch.cuda.synchronize()
            rows = []
            for _ in range(7):
                t0 = time.perf_counter()
                g.replay()
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                rows.append((t1 - t0, time.perf_counter() - t0))
            rows.sort(key=lambda r: r[1])
            h, tot = rows[len(rows) // 2]
            print(json.dumps({"case": name, "kernels": n, "replay_host_us": round(h * 1e6, 1),
                              "replay_total_us": round(tot * 1e6, 1)}), flush=True)


if __name__ == "__main__":
    import sys
    if "--ours" in sys.argv:
        ours()
    else:
        main()
