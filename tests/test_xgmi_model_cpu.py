"""The xGMI cost model behind the TP all-reduce dispatch (parallel/xgmi_model.py,
VERDICT r4 next #3d): its crossovers, and that the dispatch follows it."""
from mcp_amd.parallel import xgmi_model as xm


def test_one_shot_two_shot_crossover_by_world_size():
    # two ranks: two-shot moves the same bytes as one-shot plus a barrier
    assert xm.k12_mode(1 << 30, 2) == 1
    assert xm.one_shot_max_bytes(2) == 1 << 30
    # 8 ranks: one-shot reads the whole message on each of 7 links, two-shot
    # 2/8 of it; the extra barrier is worth ~300 KB of link time
    x8 = xm.one_shot_max_bytes(8)
    assert 250_000 < x8 < 370_000, x8
    assert xm.k12_mode(16 << 10, 8) == 1 and xm.k12_mode(4 << 20, 8) == 2
    x4 = xm.one_shot_max_bytes(4)
    assert x8 < x4 < 600_000, x4


def test_k12_beats_rccl_wherever_it_fits():
    for n in (2, 4, 8):
        for m in (8 << 10, 256 << 10, 1 << 20, 8 << 20, 64 << 20):
            path, us = xm.best(m, n, 64 << 20)
            assert path.startswith("k12"), (n, m, path)
            assert us < xm.rccl_us(m, n)
        assert xm.best(128 << 20, n, 64 << 20)[0] == "rccl"


def test_decode_and_prefill_messages_at_70b_tp8():
    """[B, 8192] bf16 decode messages go one-shot, prefill-size [T, 8192] ones
    two-shot, and a 2048-token prefill message under half RCCL's price."""
    H = 8192
    assert xm.best(8 * H * 2, 8, 64 << 20)[0] == "k12-1"
    assert xm.best(640 * H * 2, 8, 64 << 20)[0] == "k12-2"
    assert xm.two_shot_us(2048 * H * 2, 8) < 0.6 * xm.rccl_us(2048 * H * 2, 8)
