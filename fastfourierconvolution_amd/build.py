"""Build the gfx950 shared library ``libffc_amd.so`` in-tree with hipcc.

    python -m fastfourierconvolution_amd.build        # or __graft_entry__.build()

Sources: fastfourierconvolution_amd/csrc/*.hip, *.cpp.  The C ABI is include/ffc_amd.h.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libffc_amd.so")
BUILD = os.path.join(PKG, "build_obj")
ARCH = os.environ.get("FFC_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function"]


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))


def _deps_mtime():
    ts = [os.path.getmtime(os.path.join(CSRC, f)) for f in os.listdir(CSRC)]
    ts.append(os.path.getmtime(os.path.join(PKG, "..", "include", "ffc_amd.h")))
    ts.append(os.path.getmtime(__file__))
    return max(ts)


def _compile(src):
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    if os.path.exists(obj) and os.path.getmtime(obj) >= _deps_mtime():
        return obj
    cmd = [HIPCC, *FLAGS, "-c", src, "-o", obj]
    if src.endswith(".cpp"):
        cmd = [HIPCC, *FLAGS, "-x", "hip", "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= _deps_mtime():
        return LIB
    srcs = sources()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(_compile, srcs))
    tmp = LIB + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB)
    if verbose:
        print(f"built {LIB}", file=sys.stderr)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
