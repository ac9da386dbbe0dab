"""Measured GEMM tile plan (ops/gemm_plan_gfx950.json, tools/tune_gemm_plan.py):
the JSON is well formed and the kernel library's host-side selector installs
and consults it.  Host code only - runs without a GPU whenever the HIP kernel
library can be loaded (it links libamdhip64; no device call is made)."""
import json
import os

import pytest

import mcp_amd.ops as ops


def _lib():
    try:
        return ops.lib()
    except Exception as e:          # library not built / HIP runtime missing
        pytest.skip(f"kernel library not loadable: {e}")


def test_plan_file_shape():
    with open(ops.GEMM_PLAN_FILE) as f:
        plan = json.load(f)
    assert plan["arch"] == "gfx950" and plan["mstep"] == 64
    shapes = {(s["N"], s["K"]) for s in plan["shapes"]}
    # the four Llama-3-8B TP=1 projections: qkv, o, gate|up, down (+ the 70B ones, config 4)
    assert {(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)} <= shapes
    assert {(10240, 8192), (8192, 8192), (57344, 8192), (8192, 28672)} <= shapes
    for s in plan["shapes"]:
        assert all(c in (-1, 0, 1, 2, 3, 4, 5) for c in s["codes"])
        # buckets below 256 rows are left to the skinny / 128 kernels
        assert all(c == -1 for c in s["codes"][:3])
        assert all(c >= 0 for c in s["codes"][3:])


def test_no_library_route():
    """Every GEMM bucket runs on our own kernels: the plan carries no hipBLASLt
    ("lib") buckets and ops has no library dispatch."""
    with open(ops.GEMM_PLAN_FILE) as f:
        plan = json.load(f)
    assert all("lib" not in s for s in plan["shapes"])
    assert not hasattr(ops, "_lib_pick") and not hasattr(ops, "_LIB_RES")


def test_plan_lookup_buckets():
    L = _lib()
    try:
        L.gemm_plan_clear()
        assert L.gemm_plan_lookup(1000, 4096, 4096) == -1
        codes = [-1, -1, -1, 0, 1, 2, 0]
        L.gemm_plan_set(4096, 4096, codes)
        # bucket b = rows (64 b, 64 b + 64]
        assert L.gemm_plan_lookup(256, 4096, 4096) == 0        # bucket 3
        assert L.gemm_plan_lookup(257, 4096, 4096) == 1        # bucket 4
        assert L.gemm_plan_lookup(320, 4096, 4096) == 1
        assert L.gemm_plan_lookup(321, 4096, 4096) == 2
        assert L.gemm_plan_lookup(448, 4096, 4096) == 0        # last bucket
        assert L.gemm_plan_lookup(449, 4096, 4096) == -1       # past the plan
        assert L.gemm_plan_lookup(300, 4096, 14336) == -1      # other shape
        # the selector follows the plan: 0 -> 128^2 kernel, 1/2 -> AGPR kernel
        assert L.gemm_select(256, 4096, 4096) == 0
        assert L.gemm_select(300, 4096, 4096) == 1
        assert L.gemm_select(350, 4096, 4096) == 1                # 192-row code
        assert L.gemm_select(400, 4096, 4096) == 0
        L.gemm_plan_set(4096, 4096, [-1] * 8)                  # replace, not append
        assert L.gemm_plan_lookup(300, 4096, 4096) == -1
        with pytest.raises(Exception):
            L.gemm_plan_set(4096, 4096, [6])
    finally:
        L.gemm_plan_clear()
        ops._load_gemm_plan(L)


def test_plan_loader_env(tmp_path, monkeypatch):
    L = _lib()
    p = tmp_path / "plan.json"
    p.write_text(json.dumps({"arch": "gfx950", "mstep": 64,
                             "shapes": [{"N": 512, "K": 256, "codes": [-1, -1, -1, 2]}]}))
    try:
        assert ops._load_gemm_plan(L, str(p)) == 1
        assert L.gemm_plan_lookup(256, 512, 256) == 2
        assert L.gemm_plan_lookup(2600, 4096, 4096) == -1     # the default plan was replaced
        monkeypatch.setenv("MCP_GEMM_PLAN", "0")
        assert ops._load_gemm_plan(L) == 0                     # disabled: nothing installed
    finally:
        monkeypatch.delenv("MCP_GEMM_PLAN", raising=False)
        L.gemm_plan_clear()
        assert ops._load_gemm_plan(L) == len(json.load(open(ops.GEMM_PLAN_FILE))["shapes"])
    assert os.path.exists(ops.GEMM_PLAN_FILE)
