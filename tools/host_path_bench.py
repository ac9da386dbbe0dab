"""Host-side cost of the engine's step loop (schedule + pack + retire/grammar
update) with the GPU mocked out: the forward returns nothing and sampling
draws a random allowed token, so only the Python / native host path runs.
Same workload as bench.py (256 intents, 10 services, 5-node plans).

    python tools/host_path_bench.py [batches] [--profile]
"""
import cProfile
import os
import pstats
import random
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mcp_amd.engine import engine as eng  # noqa: E402
from mcp_amd.models.llama import get_config  # noqa: E402
from mcp_amd.planner.local import LocalPlanner  # noqa: E402
from mcp_amd.planner.prompt import synthetic_intent  # noqa: E402
from mcp_amd.registry import MemoryRegistry, synthetic_registry  # noqa: E402


class _Model:
    def __init__(self):
        import dataclasses
        # Llama-3-8B head layout, one layer: the KV cache only has to exist
        self.cfg = dataclasses.replace(get_config("llama3-8b"), layers=1)
        self.device = torch.device("cpu")
        self.hkv = self.cfg.kv_heads
        self.tp = 1


class MockEngine(eng.LLMEngine):
    """LLMEngine whose launch / sample never touch a device."""

    def _launch(self, host, layout):
        return None, None

    def _sample(self, hidden, dstep, n):
        return None, None

    def _retire(self, L):
        toks = [random.choice(q.decoder.allowed()) for q in L.sample_seqs]
        L.tokens = torch.tensor(toks, dtype=torch.int32) if toks else None
        super()._retire(L)


def main():
    batches = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 3
    random.seed(0)
    e = MockEngine(_Model(), num_blocks=4096, max_batch=264, max_step_tokens=4096,
                   pipeline=False, graphs=False)
    reg = MemoryRegistry(synthetic_registry(10, seed=1))
    pl = LocalPlanner(e, reg, max_nodes=5, min_nodes=5)
    pl.plan_many([synthetic_intent(-1 - i) for i in range(256)])          # warm caches
    e.stats.update({k: 0.0 for k in ("schedule_s", "update_s")})
    steps0 = e.stats["steps"]
    prof = cProfile.Profile() if "--profile" in sys.argv else None
    t = time.perf_counter()
    if prof:
        prof.enable()
    for b in range(batches):
        pl.plan_many([synthetic_intent(b * 256 + i) for i in range(256)])
    if prof:
        prof.disable()
    dt = time.perf_counter() - t
    steps = e.stats["steps"] - steps0
    print(f"{batches} batches, {steps} steps: {dt / steps * 1e3:.3f} ms host per step "
          f"(schedule {e.stats['schedule_s'] / steps * 1e3:.3f}, update {e.stats['update_s'] / steps * 1e3:.3f})")
    if prof:
        pstats.Stats(prof).sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
