"""Fold the shapes of one GEMM plan file into another (same arch / mstep):
shapes present in ``src`` replace those of ``dst``; keys of an existing shape
that ``src`` lacks (e.g. the "lib" buckets) are kept.

    python tools/merge_gemm_plan.py src.json [dst.json]
"""
import json
import os
import sys

src = json.load(open(sys.argv[1]))
dst_path = sys.argv[2] if len(sys.argv) > 2 else os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "..",
    "autonomous-microservice-composition-via-llm-agents-in-an-mcp-control-plane_amd", "ops",
    "gemm_plan_gfx950.json")
dst = json.load(open(dst_path))
assert src["arch"] == dst["arch"] and src["mstep"] == dst["mstep"]
by = {(s["N"], s["K"]): s for s in dst["shapes"]}
for s in src["shapes"]:
    old = by.get((s["N"], s["K"]), {})
    by[(s["N"], s["K"])] = {**old, **s}
dst["shapes"] = list(by.values())
for k, v in src.items():
    if k not in ("shapes", "generated"):
        dst.setdefault(k, v)
with open(dst_path, "w") as f:
    json.dump(dst, f, indent=None, separators=(",", ":"))
    f.write("\n")
print(json.dumps({"shapes": [(s["N"], s["K"]) for s in dst["shapes"]], "written": dst_path}))
