"""Every library function a GPU test, tool or the ops layer calls on the HIP
extension is bound in csrc/bindings.cpp (a missing m.def only shows up on the
GPU box, as an AttributeError)."""
import pathlib
import re

ROOT = pathlib.Path(__file__).resolve().parents[1]
PKG = next(p for p in ROOT.iterdir() if p.name.endswith("_amd") and p.is_dir())


def test_every_called_library_function_is_bound():
    bound = set(re.findall(r'm\.def\("(\w+)"', (PKG / "csrc" / "bindings.cpp").read_text()))
    srcs = list((ROOT / "tests").glob("*.py")) + list((ROOT / "tools").glob("*.py")) + \
        list((PKG / "ops").glob("*.py"))
    called = {}
    for f in srcs:
        text = f.read_text()
        names = set(re.findall(r"\bL\.(\w+)\(", text)) | set(re.findall(r"lib\(\)\.(\w+)\(", text))
        for n in names:
            called.setdefault(n, f.name)
    missing = {n: f for n, f in called.items() if n not in bound}
    assert not missing, f"called but not bound: {missing}"
