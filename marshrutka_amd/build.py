"""Builds libmarshrutka_pf.so in-tree for gfx950 (hipcc cross-compiles; no GPU
needed).  Usage: python -m marshrutka_amd.build"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB_DIR = os.path.join(HERE, "lib")
LIB_PATH = os.path.join(LIB_DIR, "libmarshrutka_pf.so")
SOURCES = ["mr_kernel.hip", "mr_host.cpp", "mr_html.cpp", "mr_render.cpp"]
HEADERS = ["mr_engine.hpp", os.path.join("..", "..", "include", "marshrutka_pf.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
         "-Wno-unused-result", "-munsafe-fp-atomics"]


def _stale() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    return any(os.path.getmtime(os.path.join(CSRC, f)) > t for f in SOURCES + HEADERS)


def build_diag(verbose: bool = False) -> str:
    """Diagnostic build with per-phase s_memtime stamps (-DMR_STAMPS) into
    lib/diag/; load it with MR_LIB_PATH=<path>.  Never used by the product path."""
    out = os.path.join(LIB_DIR, "diag", "libmarshrutka_pf.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    flag = "-DMR_HUBDUMP" if os.environ.get("MR_DIAG") == "hubdump" else "-DMR_STAMPS"
    cmd = [HIPCC, *FLAGS, flag, *[os.path.join(CSRC, s) for s in SOURCES], "-o", out]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return out


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB_PATH
    os.makedirs(LIB_DIR, exist_ok=True)
    tmp = LIB_PATH + ".tmp"
    cmd = [HIPCC, *FLAGS, *[os.path.join(CSRC, s) for s in SOURCES], "-o", tmp]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    if "--diag" in sys.argv:
        print(build_diag(verbose=True))
    else:
        build(force="--force" in sys.argv, verbose=True)
        print(LIB_PATH)
