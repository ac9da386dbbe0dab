"""utils/heap.settle: the start-up heap goes to the permanent generation and
the young-generation threshold rises; MCP_GC_SETTLE=0 keeps the defaults."""
import gc

from mcp_amd.utils import heap


def test_settle_freezes_and_raises_threshold(monkeypatch):
    old = gc.get_threshold()
    try:
        monkeypatch.setenv("MCP_GC_GEN0", "12345")
        keep = [[i] for i in range(100)]           # long-lived start-up objects
        assert heap.settle()
        assert gc.get_threshold()[0] == 12345
        assert gc.get_freeze_count() >= len(keep)
        monkeypatch.setenv("MCP_GC_SETTLE", "0")
        gc.set_threshold(*old)
        assert not heap.settle()
        assert gc.get_threshold() == old
    finally:
        gc.unfreeze()
        gc.set_threshold(*old)
