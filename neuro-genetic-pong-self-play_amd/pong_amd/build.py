"""Build ``libpong_ga.so`` in-tree with hipcc for gfx950 (no JIT cache: the
.so travels with the repository snapshot to the GPU box)."""
from __future__ import annotations

import os
import subprocess
import sys

from ._lib import LIB_PATH, PKG_DIR, REPO_DIR

CSRC = os.path.join(PKG_DIR, "csrc")
HEADERS = [os.path.join(CSRC, h) for h in ("pg_device.hpp", "pg_f64math.h", "pg_eval.hpp", "pg_cascade.hpp",
                                           "pg_service.hpp")] + [os.path.join(REPO_DIR, "include", "pong_ga.h")]
# one translation unit per kernel family, compiled in parallel and linked into one .so;
# pg_service_more.hip is compiled once per (lanes per game, genome type): its ~100
# k_service instantiations took 10 minutes as one unit
# (object name, source, extra flags)
UNITS = [("pong_ga", "pong_ga.hip", []), ("pg_wide", "pg_wide.hip", []), ("pg_pixels", "pg_pixels.hip", []),
         ("pg_hof", "pg_hof.hip", []), ("pg_gen", "pg_gen.hip", []), ("pg_decide", "pg_decide.hip", [])] + [
    (f"pg_service_more_L{L}_{f}", "pg_service_more.hip",
     [f"-DPG_MORE_L={L}", f"-DPG_MORE_F64={f}"] + (["-DPG_MORE_DISPATCH"] if (L, f) == (8, 1) else []))
    for L in (8, 16, 32, 64) for f in (1, 0)]
SOURCES = sorted({os.path.join(CSRC, src) for _, src, _ in UNITS})
DEPS = SOURCES + [os.path.abspath(__file__)] + HEADERS
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# per-source flags: the iterative ILP machine scheduler makes k_service's frame
# loop ~5 % faster on the bench than the default (13.57 vs 14.3 ms per launch;
# max-ilp 13.85; iterative-minreg +9 %, max-memory-clause +4 %,
# iterative-maxocc +37 %, the newer RP trackers +6 %, -O2 +3 % slower)
# (pg_service_more.hip keeps the default scheduler: iterative-ilp crashes the
# register allocator on some small k_service layouts in this compiler, so
# pong_ga.hip instantiates only the bench layout)
SOURCE_FLAGS = {"pong_ga.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]}
ARCH = os.environ.get("PG_OFFLOAD_ARCH", "gfx950")


def _obj(name: str) -> str:
    return os.path.join(CSRC, name + ".o")


def _flags() -> list:
    return [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-ffp-contract=off"] + [
        # no SLP packing of independent f32 adds into v_pk_add_f32: it breaks the
        # DPP-fused reductions into mov_dpp + pk_add pairs (measured -5 %)
        "-fno-slp-vectorize", "-fPIC",
        "-Wall", "-Wno-unused-function", "-I", os.path.join(REPO_DIR, "include")]


def _unit_cmd(src: str, extra: list, out: str) -> list:
    return [HIPCC] + _flags() + SOURCE_FLAGS.get(os.path.basename(src), []) + extra + ["-c", "-o", out, src]


def _link_cmd(objs: list, out: str) -> list:
    return [HIPCC, f"--offload-arch={ARCH}", "-shared", "-o", out] + sorted(objs)


def _read(path: str):
    try:
        with open(path) as fh:
            return fh.read()
    except OSError:
        return None


def _write(path: str, text: str) -> None:
    with open(path + ".tmp", "w") as fh:
        fh.write(text)
    os.replace(path + ".tmp", path)


# Stamps: each object's compile command and the content hash of its inputs
# (the source, every shared header, this file), and the library's whole recipe,
# written next to them.  A build input that is not a file -- PG_OFFLOAD_ARCH,
# HIPCC, the flags above -- changes the command, so an object or library built
# with another one is rebuilt, not linked into a library labelled with the new
# arch (round-5 review).  Paths are stamped relative to the repository and
# inputs by content, not mtime: a copy of the tree elsewhere (the GPU box's
# snapshot) finds its prebuilt library current instead of rebuilding it.
def _rel(cmd: list) -> str:
    return " ".join(cmd).replace(REPO_DIR, "<repo>")


def _digest(paths: list) -> str:
    import hashlib
    h = hashlib.sha256()
    for path in paths:
        with open(path, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:32]


def _unit_stamp(name: str, src: str, extra: list) -> str:
    inputs = [os.path.join(CSRC, src), os.path.abspath(__file__)] + HEADERS
    return _rel(_unit_cmd(os.path.join(CSRC, src), extra, _obj(name))) + " #" + _digest(inputs)


def _lib_stamp() -> str:
    lines = [_unit_stamp(name, src, extra) for name, src, extra in sorted(UNITS)]
    lines.append(_rel(_link_cmd([_obj(name) for name, _, _ in UNITS], LIB_PATH)))
    return "\n".join(lines) + "\n"


def _stale(name: str, src: str, extra: list) -> bool:
    """An object is rebuilt when it is missing or its stamp differs: another
    command, or another content of its source, any shared header or this file
    (headers are not tracked per unit)."""
    obj = _obj(name)
    return not os.path.exists(obj) or _read(obj + ".stamp") != _unit_stamp(name, src, extra)


def needs_build() -> bool:
    return not os.path.exists(LIB_PATH) or _read(LIB_PATH + ".stamp") != _lib_stamp()


def build(force: bool = False, verbose: bool = False) -> str:
    if os.environ.get("PONG_GA_LIB") and not force:
        return LIB_PATH  # a prebuilt variant (tools/build_variant.py): never rebuilt from the product sources
    if not force and not needs_build():
        return LIB_PATH
    objs, procs = [], []
    # the slow units first, so the parallel build ends sooner
    for name, src, extra in sorted(UNITS, key=lambda u: not u[0].startswith("pg_service_more")):
        obj = _obj(name)
        objs.append(obj)
        if not force and not _stale(name, src, extra):
            continue
        cmd = _unit_cmd(os.path.join(CSRC, src), extra, obj + ".tmp")
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((subprocess.Popen(cmd), cmd, obj, _unit_stamp(name, src, extra)))
    for proc, cmd, obj, stamp in procs:
        if proc.wait() != 0:
            raise subprocess.CalledProcessError(proc.returncode, cmd)
        os.replace(obj + ".tmp", obj)
        _write(obj + ".stamp", stamp)
    link = _link_cmd(objs, LIB_PATH + ".tmp")
    if verbose:
        print(" ".join(link), file=sys.stderr)
    subprocess.check_call(link)
    os.replace(LIB_PATH + ".tmp", LIB_PATH)
    _write(LIB_PATH + ".stamp", _lib_stamp())
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
