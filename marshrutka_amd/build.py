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
# one translation unit per kernel family (device code shared through mr_device.hpp),
# compiled in parallel and linked into one shared library
SOURCES = ["mr_k_region.hip", "mr_k_groupq.hip", "mr_k_group.hip", "mr_k_group_nl.hip", "mr_k_lane.hip", "mr_k_lane24.hip", "mr_k_lane32.hip", "mr_k_lane_nl.hip", "mr_k_lane_nl2.hip", "mr_k_wide2.hip", "mr_k_wide5.hip", "mr_k_wide8.hip", "mr_k_hub_lin.hip", "mr_k_hub_nl.hip",
           "mr_k_hub.hip", "mr_k_wide.hip",
           "mr_k_solve.hip", "mr_k_fill.hip", "mr_k_cert.hip", "mr_k_decode.hip",
           "mr_host.cpp", "mr_html.cpp", "mr_render.cpp"]
HEADERS = ["mr_engine.hpp", "mr_pool.hpp", "mr_device.hpp", "mr_hub_lane.hpp", "mr_hub_group.hpp", "mr_cert.hpp", "mr_cert_tile.hpp", os.path.join("..", "..", "include", "marshrutka_pf.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall",
         "-Wno-unused-result", "-munsafe-fp-atomics"]


def _compile_link(out: str, extra: list, verbose: bool) -> None:
    """Compiles every source to an object (in parallel) and links `out`."""
    from concurrent.futures import ThreadPoolExecutor
    obj_dir = os.path.join(os.path.dirname(out), "obj" + ("_" + "_".join(x.strip("-") for x in extra) if extra else ""))
    os.makedirs(obj_dir, exist_ok=True)

    def one(src: str) -> str:
        obj = os.path.join(obj_dir, os.path.splitext(src)[0] + ".o")
        cmd = [HIPCC, *FLAGS, *extra, "-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        return obj

    jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(one, SOURCES))
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", out]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


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
    _compile_link(out, [flag], verbose)
    return out


def build_variant(tag: str, defines: list, verbose: bool = False) -> str:
    """Experiment build with extra -D flags into lib/variants/<tag>/ (A/B runs load it
    with MR_LIB_PATH=<path>).  Never used by the product path."""
    out = os.path.join(LIB_DIR, "variants", tag, "libmarshrutka_pf.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    _compile_link(out, list(defines), verbose)
    return out


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB_PATH
    os.makedirs(LIB_DIR, exist_ok=True)
    tmp = LIB_PATH + ".tmp"
    _compile_link(tmp, [], verbose)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    if "--diag" in sys.argv:
        print(build_diag(verbose=True))
    elif "--variant" in sys.argv:  # --variant TAG -DNAME=V ...
        i = sys.argv.index("--variant")
        print(build_variant(sys.argv[i + 1], [a for a in sys.argv[i + 2:] if a.startswith("-D")], verbose=False))
    else:
        build(force="--force" in sys.argv, verbose=True)
        print(LIB_PATH)
