"""Cyclic-GC settings for a serving process after start-up.

Everything built at start-up (model and graph objects, registry, tokenizer
tables, compiled grammars) lives for the whole process.  CPython's cyclic
collector would keep rescanning it: with the default thresholds a planner
process runs ~25 young collections per engine step and a gen-1 pass every
~10 of those (~1 ms each on the 256-intent headline batch, measured with
``gc.callbacks`` over ``bench.py --device cpu --model tiny``), all on the
thread that launches the GPU work.  ``settle()`` moves the start-up heap to
the permanent generation (``gc.freeze``) and raises the young-generation
threshold so the per-step garbage, which reference counting already frees,
no longer triggers scans.  Cycles are still collected, just less often.

``MCP_GC_SETTLE=0`` keeps CPython's defaults; ``MCP_GC_GEN0`` sets the
young threshold (default 50000 allocations).
"""
import gc
import os


def settle() -> bool:
    """Freeze the start-up heap and raise the young-generation threshold;
    False when disabled."""
    if os.environ.get("MCP_GC_SETTLE", "1") != "1":
        return False
    gc.collect()
    gc.freeze()
    gen0 = int(os.environ.get("MCP_GC_GEN0", "50000"))
    _, g1, g2 = gc.get_threshold()
    gc.set_threshold(max(gen0, 1), g1, g2)
    return True
