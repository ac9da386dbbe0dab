"""The shipped GEMM plan (ops/gemm_plan_gfx950.json) holds measured entries
for every projection shape the planner runs: Llama-3 8B and 70B at TP 1, 2,
4 and 8 (Megatron 1-D shards, tools/tune_gemm_plan.py shard_shapes)."""
import json
import pathlib

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
PKG = next(p for p in ROOT.iterdir() if p.name.endswith("_amd") and p.is_dir())
ARCH = {"8b": (4096, 32, 8, 14336), "70b": (8192, 64, 8, 28672)}


def shard_shapes(name, t):
    H, hq, hkv, F = ARCH[name]
    return [((hq + 2 * hkv) * 128 // t, H), (H, hq * 128 // t), (2 * F // t, H), (H, F // t)]


@pytest.mark.parametrize("model", ["8b", "70b"])
@pytest.mark.parametrize("tp", [1, 2, 4, 8])
def test_plan_covers_every_shard_shape(model, tp):
    plan = json.loads((PKG / "ops" / "gemm_plan_gfx950.json").read_text())
    have = {(s["N"], s["K"]): s for s in plan["shapes"]}
    for nk in shard_shapes(model, tp):
        assert nk in have, (model, tp, nk)
        codes = have[nk]["codes"]
        assert len(codes) >= 64 and all(-1 <= c <= 5 for c in codes)


def test_merge_keys_folds_only_named_buckets(tmp_path):
    """tools/merge_gemm_plan.py --keys flex: a short source (the buckets it
    measured) overwrites that key's prefix in the destination shape and leaves
    every other key and bucket alone; a shape missing from dst is an error."""
    import subprocess
    import sys
    tool = pathlib.Path(__file__).resolve().parents[1] / "tools" / "merge_gemm_plan.py"
    dst = {"arch": "gfx950", "mstep": 64, "shapes": [
        {"N": 64, "K": 64, "codes": [1, 2, 3, 4], "splits": [0, 0, 0, 0], "flex": [-1, -1, 5, 6]}]}
    src = {"arch": "gfx950", "mstep": 64, "generated": "x", "shapes": [
        {"N": 64, "K": 64, "codes": [9, 9], "splits": [8, 8], "flex": [7, -1]}]}
    d, s = tmp_path / "dst.json", tmp_path / "src.json"
    d.write_text(json.dumps(dst))
    s.write_text(json.dumps(src))
    subprocess.run([sys.executable, str(tool), str(s), str(d), "--keys", "flex"], check=True,
                   capture_output=True)
    out = json.loads(d.read_text())["shapes"][0]
    assert out["flex"] == [7, -1, 5, 6]
    assert out["codes"] == [1, 2, 3, 4] and out["splits"] == [0, 0, 0, 0]
    src["shapes"][0]["N"] = 128
    s.write_text(json.dumps(src))
    r = subprocess.run([sys.executable, str(tool), str(s), str(d), "--keys", "flex"],
                       capture_output=True)
    assert r.returncode != 0
