"""Build ``libpong_ga.so`` in-tree with hipcc for gfx950 (no JIT cache: the
.so travels with the repository snapshot to the GPU box)."""
from __future__ import annotations

import os
import subprocess
import sys

from ._lib import LIB_PATH, PKG_DIR, REPO_DIR

SOURCES = [os.path.join(PKG_DIR, "csrc", "pong_ga.hip")]
DEPS = SOURCES + [os.path.abspath(__file__), os.path.join(PKG_DIR, "csrc", "pg_device.hpp"), os.path.join(PKG_DIR, "csrc", "pg_f64math.h"),
        os.path.join(REPO_DIR, "include", "pong_ga.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PG_OFFLOAD_ARCH", "gfx950")


def needs_build() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    return any(os.path.getmtime(d) > t for d in DEPS)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return LIB_PATH
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-ffp-contract=off",
           # no SLP packing of independent f32 adds into v_pk_add_f32: it breaks the
           # DPP-fused reductions into mov_dpp + pk_add pairs (measured -5 %)
           "-fno-slp-vectorize", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function", "-I", os.path.join(REPO_DIR, "include"),
           "-o", LIB_PATH + ".tmp"] + SOURCES
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(LIB_PATH + ".tmp", LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
