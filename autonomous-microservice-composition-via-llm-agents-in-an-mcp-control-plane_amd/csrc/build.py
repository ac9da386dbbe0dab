"""In-tree build of the gfx950 kernel library and the native runtime.

    python csrc/build.py [--force] [--jobs N] [--verbose]

* every ``*.hip`` file is compiled separately by ``hipcc --offload-arch=gfx950``
  (no torch headers -> seconds per file);
* ``bindings.cpp`` (pybind11 + ATen) is compiled once by the host compiler;
* everything links into ``ops/_kernels<EXT_SUFFIX>`` next to the Python
  wrappers, so the ``.so`` travels with the repo snapshot to the GPU box.
* ``runtime/*.cpp`` (CPU-side native runtime: paged-KV block allocator, grammar
  mask builder) links into ``engine/_runtime<EXT_SUFFIX>``.

Incremental: an object is rebuilt only when a source or header is newer.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
PKG = HERE.parent
BUILD = HERE / "build"
ARCH = os.environ.get("MCP_OFFLOAD_ARCH", "gfx950")
EXT = sysconfig.get_config_var("EXT_SUFFIX")
KERNELS_SO = PKG / "ops" / f"_kernels{EXT}"
RUNTIME_SO = PKG / "engine" / f"_runtime{EXT}"


def _torch_paths():
    import torch
    root = Path(torch.__file__).resolve().parent
    return root / "include", root / "lib"


def _py_includes():
    import pybind11
    return [sysconfig.get_paths()["include"], pybind11.get_include()]


def _newer(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(map(str, cmd)), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"command failed: {cmd[0]} ... {cmd[-1]}")
    if verbose and (r.stdout or r.stderr):
        sys.stderr.write(r.stdout + r.stderr)


def build(force: bool = False, jobs: int = 8, verbose: bool = False) -> Path:
    BUILD.mkdir(exist_ok=True)
    headers = list(HERE.glob("*.h"))
    tinc, tlib = _torch_paths()
    hip_srcs = sorted(HERE.glob("*.hip"))
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    cxx = shutil.which("g++") or "g++"
    common_hip = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
                  "-ffp-contract=fast", "-munsafe-fp-atomics", f"-I{HERE}"]
    jobs_list = []
    objs = []
    for src in hip_srcs:
        obj = BUILD / (src.stem + ".o")
        objs.append(obj)
        if force or _newer(obj, [src] + headers):
            jobs_list.append([*common_hip, "-c", str(src), "-o", str(obj)])
    bsrc = HERE / "bindings.cpp"
    bobj = BUILD / "bindings.o"
    objs.append(bobj)
    if force or _newer(bobj, [bsrc] + headers):
        jobs_list.append([cxx, "-O2", "-std=c++17", "-fPIC", "-D__HIP_PLATFORM_AMD__", "-DUSE_ROCM",
                          "-DTORCH_EXTENSION_NAME=_kernels", "-DTORCH_API_INCLUDE_EXTENSION_H",
                          "-D_GLIBCXX_USE_CXX11_ABI=1", f"-I{HERE}", f"-I{tinc}",
                          f"-I{tinc / 'torch/csrc/api/include'}", "-I/opt/rocm/include",
                          *[f"-I{p}" for p in _py_includes()], "-c", str(bsrc), "-o", str(bobj)])
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs_list))
    if force or jobs_list or not KERNELS_SO.exists():
        _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o",
              str(KERNELS_SO), f"-L{tlib}", "-ltorch", "-ltorch_cpu", "-lc10", "-lc10_hip",
              "-ltorch_hip", "-ltorch_python", "-L/opt/rocm/lib", "-lrccl", f"-Wl,-rpath,{tlib}",
              "-Wl,-rpath,/opt/rocm/lib"], verbose)
    _check_stubs(KERNELS_SO)
    build_runtime(force, verbose)
    return KERNELS_SO


def _check_stubs(so: Path) -> None:
    """Fail the build when a kernel's host launch stub is missing from the
    library: hipcc's host pass silently drops the stub of a kernel whose body
    it rejects (e.g. a class local to the kernel used by its lambdas), and the
    library then fails only at load time on the GPU box."""
    nm = shutil.which("nm")
    if not nm:
        return
    r = subprocess.run([nm, "-D", "--undefined-only", str(so)], capture_output=True, text=True)
    missing = [ln.split()[-1] for ln in r.stdout.splitlines() if "__device_stub__" in ln]
    if missing:
        raise RuntimeError(f"{so.name}: {len(missing)} kernel launch stubs undefined, e.g. {missing[0]}")


def build_runtime(force: bool = False, verbose: bool = False) -> Path | None:
    rdir = HERE / "runtime"
    srcs = sorted(rdir.glob("*.cpp")) if rdir.exists() else []
    if not srcs:
        return None
    deps = srcs + list(rdir.glob("*.h"))
    if force or _newer(RUNTIME_SO, deps):
        cxx = shutil.which("g++") or "g++"
        _run([cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-DMODULE_NAME=_runtime",
              *[f"-I{p}" for p in _py_includes()], *map(str, srcs), "-o", str(RUNTIME_SO)], verbose)
    return RUNTIME_SO


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args()
    print(build(a.force, a.jobs, a.verbose))
