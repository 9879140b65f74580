"""Builds the in-tree HIP extension ``mtl_das_pytorch_amd/_mda_hip*.so`` with hipcc for gfx950 only.

No torch C++ headers and no hipify step: the kernels are plain HIP C++ and the bindings use pybind11,
so a full rebuild takes a few seconds per translation unit.  Objects are compiled in parallel; a
translation unit is recompiled when it or any header is newer than its object (``--force``: all of them).

    python -m mtl_das_pytorch_amd.csrc.build [--force] [--debug]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ARCH = os.environ.get("MDA_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def so_path() -> str:
    return os.path.join(PKG, "_mda_hip" + sysconfig.get_config_var("EXT_SUFFIX"))


def _sources():
    return (sorted(glob.glob(os.path.join(HERE, "*.hip"))) + [os.path.join(HERE, "bindings.cpp")]
            + [os.path.join(HERE, "matio.cpp")])


def needs_build() -> bool:
    so = so_path()
    if not os.path.exists(so):
        return True
    t = os.path.getmtime(so)
    deps = _sources() + glob.glob(os.path.join(HERE, "*.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, debug: bool = False, verbose: bool = True, jobs: int = 8) -> str:
    so = so_path()
    if not force and not needs_build():
        return so
    import pybind11
    obj_dir = os.path.join(HERE, "build")
    os.makedirs(obj_dir, exist_ok=True)
    common = ["--offload-arch=" + ARCH, "-fPIC", "-std=c++17", "-O1" if debug else "-O3",
              "-I" + HERE, "-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"],
              "-Wno-unused-result", "-Wno-unused-variable"]
    if debug:
        common += ["-g"]

    headers = glob.glob(os.path.join(HERE, "*.h"))
    newest_dep = max([os.path.getmtime(h) for h in headers] + [os.path.getmtime(__file__)])

    def compile_one(src):
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        if not force and os.path.exists(obj) and os.path.getmtime(obj) > max(os.path.getmtime(src), newest_dep):
            return obj  # incremental: this translation unit and every header are older than its object
        cmd = [HIPCC] + common + ["-c", src, "-o", obj]
        if src.endswith("bindings.cpp"):
            cmd = [HIPCC] + common + ["-x", "hip", "-c", src, "-o", obj]
        elif src.endswith(".cpp"):  # host-only C++ (native data loader): no device code objects
            cmd = [HIPCC] + [c for c in common if not c.startswith("--offload-arch")] + ["-x", "c++", "-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
        if verbose and r.stderr.strip():
            print(r.stderr, file=sys.stderr)
        return obj

    srcs = _sources()
    with cf.ThreadPoolExecutor(max_workers=min(jobs, len(srcs))) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = so + ".tmp"
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", tmp] + objs + ["-lz", "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, so)
    if verbose:
        print(f"built {so}", file=sys.stderr)
    return so


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    args = ap.parse_args()
    build(force=args.force, debug=args.debug)
