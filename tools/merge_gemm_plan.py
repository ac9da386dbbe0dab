"""Fold the shapes of one GEMM plan file into another (same arch / mstep):
shapes present in ``src`` replace those of ``dst``; keys of an existing shape
that ``src`` lacks (e.g. the "lib" buckets) are kept.

    python tools/merge_gemm_plan.py src.json [dst.json] [--keys flex,...]

``--keys``: fold only those per-bucket arrays, bucket by bucket over the
buckets ``src`` measured (a short ``src`` overwrites the prefix), keeping every
other key of ``dst``.
"""
import json
import os
import sys

args = sys.argv[1:]
keys = None
if "--keys" in args:
    i = args.index("--keys")
    keys = args[i + 1].split(",")
    del args[i:i + 2]
src = json.load(open(args[0]))
dst_path = args[1] if len(args) > 1 else os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "..",
    "autonomous-microservice-composition-via-llm-agents-in-an-mcp-control-plane_amd", "ops",
    "gemm_plan_gfx950.json")
dst = json.load(open(dst_path))
assert src["arch"] == dst["arch"] and src["mstep"] == dst["mstep"]
by = {(s["N"], s["K"]): s for s in dst["shapes"]}
for s in src["shapes"]:
    old = by.get((s["N"], s["K"]), {})
    if keys is None:
        by[(s["N"], s["K"])] = {**old, **s}
        continue
    assert old, f"--keys needs the shape in dst: {(s['N'], s['K'])}"
    for k in keys:
        cur = list(old.get(k, [-1] * len(old["codes"])))
        cur[:len(s[k])] = s[k]
        old[k] = cur
dst["shapes"] = list(by.values())
for k, v in src.items():
    if k not in ("shapes", "generated"):
        dst.setdefault(k, v)
with open(dst_path, "w") as f:
    json.dump(dst, f, indent=None, separators=(",", ":"))
    f.write("\n")
print(json.dumps({"shapes": [(s["N"], s["K"]) for s in dst["shapes"]], "written": dst_path}))
