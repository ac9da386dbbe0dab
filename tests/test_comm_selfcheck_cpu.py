"""K12 start-up self-check decision (parallel.comm.selfcheck_decision), on
CPU with simulated collectives: K12 stays on only when every rank's one-shot
and two-shot probes equal the exact sum; an injected mismatch on one rank, or
a mismatch another rank reports, turns it off everywhere with the reason; a
wrong reference (RCCL) path is flagged as an error, not silently used."""
import torch

from mcp_amd.parallel.comm import probe_values, selfcheck_decision

WORLD = 4


def _exact(n):
    return sum(probe_values(n, r, "cpu").float() for r in range(WORLD))


def _run(rank=0, inject=False, other_bad=(), ref_wrong=False):
    def custom(t, mode):
        return _exact(t.numel()).to(t.dtype)

    def reference(t):
        t.copy_(_exact(t.numel()).to(t.dtype))
        if ref_wrong:
            t[0] += 1

    def agree(mine):
        return [mine] + [{"bad": list(other_bad), "ref_bad": []}] * (WORLD - 1)
    return selfcheck_decision(rank, WORLD, [4096, 1 << 16], lambda n, r: probe_values(n, r, "cpu"),
                              custom, reference, agree, inject=inject)


def test_probe_sums_are_exact_in_bf16():
    for n in (4096, 1 << 16):
        s = _exact(n)
        assert torch.equal(s.to(torch.bfloat16).float(), s) and s.max() <= 8 * 13
        assert not torch.equal(probe_values(n, 0, "cpu"), probe_values(n, 1, "cpu"))


def test_selfcheck_keeps_k12_when_every_rank_matches():
    v = _run()
    assert v["custom_ok"] and not v["reference_error"] and v["why"] is None


def test_selfcheck_injected_mismatch_disables_k12_with_a_reason():
    v = _run(inject=True)
    assert not v["custom_ok"] and "K12 mode 1" in v["why"] and "K12 mode 2" in v["why"]
    v = _run(other_bad=["rank 2: K12 mode 2, 2097152 B: 5 wrong elements"])
    assert not v["custom_ok"] and "rank 2" in v["why"]


def test_selfcheck_flags_a_wrong_reference_path():
    v = _run(ref_wrong=True)
    assert v["reference_error"] and v["custom_ok"]
