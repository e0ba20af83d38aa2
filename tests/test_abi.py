"""The C-ABI boundary (include/pong_ga.h) without a GPU: the library loads,
exports every declared entry point, the ctypes structures match the C layout
byte for byte, and argument validation fails loudly before any HIP call."""
import ctypes
import os
import re
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "pong_ga.h")


@pytest.fixture(scope="module")
def lib():
    from pong_amd import _lib
    from pong_amd import build as B
    B.build()
    return _lib.lib()


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?(?:char|int32_t|size_t)\s*\*?\s*(pg_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_expected_entry_points():
    names = declared_functions()
    for must in ("pg_eval_population", "pg_forward", "pg_physics_step", "pg_physics_reset",
                 "pg_last_error", "pg_version", "pg_ga_vary", "pg_ga_select_tournament"):
        assert must in names


def test_library_exports_every_declared_symbol(lib):
    from pong_amd import _lib
    names = declared_functions()
    for name in names:
        assert hasattr(lib, name), f"{name} missing from {_lib.LIB_PATH}"
    assert sorted(_lib.SIGNATURES) == names, "ctypes signatures out of sync with the header"
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (pg_\w+)", out))
    assert set(names) <= exported


def test_version_and_gene_count(lib):
    from pong_amd import _lib
    assert lib.pg_abi_version() == _lib.PG_ABI_VERSION
    assert b"gfx950" in lib.pg_version()
    for shape, genes in (([6, 2, 2], 20), ([6, 64, 3], 643), ([6, 512, 512, 3], 267779)):
        net = _lib.make_net(shape)
        assert lib.pg_gene_count(ctypes.byref(net)) == genes


def test_validation_errors_without_gpu(lib):
    from pong_amd import _lib
    assert lib.pg_eval_population(None, None) == _lib.PG_ERR_INVALID
    assert b"NULL" in lib.pg_last_error()
    a = _lib.PgEvalArgs()
    a.net = _lib.make_net([5, 2, 2])
    a.n_games = 6
    assert lib.pg_eval_population(ctypes.byref(a), None) == _lib.PG_ERR_INVALID
    assert b"6 inputs" in lib.pg_last_error()
    a.net = _lib.make_net([6, 2, 2])
    a.n_games = 0
    assert lib.pg_eval_population(ctypes.byref(a), None) == _lib.PG_ERR_INVALID
    a.n_games = 6
    a.n_genomes = 0  # empty batch: nothing to do, no device touched
    assert lib.pg_eval_population(ctypes.byref(a), None) == _lib.PG_OK
    a.n_genomes = 4
    a.genome_stride = 3  # < 20 genes
    assert lib.pg_eval_population(ctypes.byref(a), None) == _lib.PG_ERR_INVALID
    assert b"genome_stride" in lib.pg_last_error()
    a.horizon = -1  # the fixed-horizon mode: T >= 0
    assert lib.pg_eval_population(ctypes.byref(a), None) == _lib.PG_ERR_INVALID
    assert b"horizon" in lib.pg_last_error()
    a.horizon = 0
    bad = _lib.make_net([6, 2, 2])
    bad.n_nodes = 1
    assert lib.pg_gene_count(ctypes.byref(bad)) == _lib.PG_ERR_INVALID
    assert lib.pg_physics_step(None, -1, None, None) == _lib.PG_ERR_INVALID


def test_workspace_bytes_follow_the_resolved_kernel(lib):
    """pg_eval_workspace_bytes sizes the kernel the arguments resolve to (host
    only, no device: the CU count falls back to 256 without a GPU): the
    general kernel needs the base (game counter + per-game flags), the split
    kernel adds its lane records (k_prep_records: one per genome and per
    opponent row, L/2 = 4 lanes x 164 f32 for [6,64,3]), the wide kernel
    adds min(n_genomes, CUs) blocks x 7 tile-major W2 copies (config 5 in f32:
    1 056 768 B per copy, its tail piece block included), and AUTO resolves
    like the launch does."""
    from pong_amd import _lib
    a = _lib.PgEvalArgs()
    a.n_games = 6
    a.n_genomes = 4096
    a.kernel = _lib.PG_KERNEL_AUTO
    base = 256 + (4096 * 6 * 4 + 255) // 256 * 256
    a.net = _lib.make_net([6, 64, 3])
    rec = 4 * 164 * 4  # 4 lanes x rec_floats<16, 3>() x 4 B per network
    assert lib.pg_eval_workspace_bytes(ctypes.byref(a)) == base + (4096 * rec + 255) // 256 * 256
    a.opponents, a.n_opponents = 1, 1024  # (a non-NULL pointer: sizing only)
    assert lib.pg_eval_workspace_bytes(ctypes.byref(a)) == base + ((4096 + 1024) * rec + 255) // 256 * 256
    a.opponents, a.n_opponents = None, 0
    a.net = _lib.make_net([6, 512, 512, 3])  # f32 (dtype 0) -> k_wide
    a.net.dtype = _lib.PG_F32
    cus = 256
    per_copy = (16 * 8 + 1) * 512 * 16  # 16 tiles x 8 pieces + 1 tail piece block, 512 rows x 16 B
    assert per_copy == 1056768
    wide = base + (min(4096, cus) * 7 * per_copy + 255) // 256 * 256
    assert lib.pg_eval_workspace_bytes(ctypes.byref(a)) == wide
    a.kernel = _lib.PG_KERNEL_GENERAL
    assert lib.pg_eval_workspace_bytes(ctypes.byref(a)) == base
    a.kernel = _lib.PG_KERNEL_WIDE
    a.n_genomes = 3  # fewer genomes than CUs: one block each
    base3 = 256 + (3 * 6 * 4 + 255) // 256 * 256
    assert lib.pg_eval_workspace_bytes(ctypes.byref(a)) == base3 + (3 * 7 * per_copy + 255) // 256 * 256
    a.n_games = 8  # more than six games: two work items (chunks of 4) per genome, a block each
    base38 = 256 + (3 * 8 * 4 + 255) // 256 * 256
    assert lib.pg_eval_workspace_bytes(ctypes.byref(a)) == base38 + (6 * 7 * per_copy + 255) // 256 * 256


def test_struct_layout_matches_c(tmp_path):
    """offsetof/sizeof of every ABI struct from gcc vs the ctypes mirror."""
    from pong_amd import _lib
    structs = {"pg_net": _lib.PgNet, "pg_eval_args": _lib.PgEvalArgs, "pg_forward_args": _lib.PgForwardArgs,
               "pg_ga_args": _lib.PgGaArgs, "pg_select_args": _lib.PgSelectArgs,
               "pg_schedule_args": _lib.PgScheduleArgs, "pg_hof_args": _lib.PgHofArgs,
               "pg_hof_rank_args": _lib.PgHofRankArgs, "pg_hof_prepare_args": _lib.PgHofPrepareArgs}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for cname, cls in structs.items():
        lines.append(f'  printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in cls._fields_:
            lines.append(f'  printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("  return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-std=c11", "-o", str(exe), str(src)])
    c = {}
    for line in subprocess.check_output([str(exe)], text=True).splitlines():
        s, f, v = line.split()
        c[(s, f)] = int(v)
    for cname, cls in structs.items():
        assert c[(cname, "size")] == ctypes.sizeof(cls), cname
        for fname, _ in cls._fields_:
            assert c[(cname, fname)] == getattr(cls, fname).offset, f"{cname}.{fname}"


def test_no_cpu_fallback_when_library_missing(tmp_path, monkeypatch):
    """The product path refuses to run without the HIP library."""
    code = ("import sys; sys.path.insert(0, %r); from pong_amd import _lib; _lib.LIB_PATH = %r; "
            "\ntry:\n    _lib.lib()\nexcept RuntimeError as e:\n    print('refused', e)" %
            (os.path.join(REPO, "neuro-genetic-pong-self-play_amd"), str(tmp_path / "missing.so")))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True)
    assert "refused" in out.stdout and "no CPU fallback" in out.stdout


def test_struct_size_refuses_other_layouts(lib):
    """ABI 10+: pg_eval_args.struct_size must be this header's sizeof; a short
    (or long) struct is refused before any other field is read, and so is the
    ABI-9 layout, whose first word (net.n_nodes) lands in struct_size."""
    from pong_amd import _lib
    a = _lib.PgEvalArgs()
    assert a.struct_size == ctypes.sizeof(_lib.PgEvalArgs)
    a.net = _lib.make_net([6, 2, 2])
    a.n_games, a.n_genomes = 6, 0
    assert lib.pg_eval_population(ctypes.byref(a), None) == _lib.PG_OK
    for size in (ctypes.sizeof(_lib.PgEvalArgs) - 8, ctypes.sizeof(_lib.PgEvalArgs) + 8, 0):
        a.struct_size = size
        assert lib.pg_eval_population(ctypes.byref(a), None) == _lib.PG_ERR_INVALID
        assert b"struct_size" in lib.pg_last_error()
        assert lib.pg_eval_workspace_bytes(ctypes.byref(a)) == 0

    class Abi10(ctypes.Structure):  # round 5's layout: ends at horizon (no episode limits)
        _fields_ = [f for f in _lib.PgEvalArgs._fields_ if f[0] not in ("timeout_thresh", "win_score")]
    a10 = Abi10()
    a10.struct_size = ctypes.sizeof(Abi10)
    a10.net = _lib.make_net([6, 2, 2])
    a10.n_games, a10.n_genomes = 6, 0
    rc = lib.pg_eval_population(ctypes.cast(ctypes.byref(a10), ctypes.POINTER(_lib.PgEvalArgs)), None)
    assert rc == _lib.PG_ERR_INVALID and b"struct_size" in lib.pg_last_error()

    class Abi9(ctypes.Structure):  # round 4's layout: no struct_size, ends at horizon
        _fields_ = [f for f in Abi10._fields_ if f[0] != "struct_size"]
    old = Abi9()
    old.net = _lib.make_net([6, 64, 3])
    old.n_games, old.n_genomes = 6, 0
    rc = lib.pg_eval_population(ctypes.cast(ctypes.byref(old), ctypes.POINTER(_lib.PgEvalArgs)), None)
    assert rc == _lib.PG_ERR_INVALID and b"struct_size=3" in lib.pg_last_error()


def test_build_stamps_are_relocatable(tmp_path):
    """The library's build stamp names no absolute path and no mtime: a copy
    of the tree elsewhere (the GPU box's snapshot, without the objects) finds
    its prebuilt libpong_ga.so current and loads it instead of rebuilding."""
    import shutil
    from pong_amd import _lib, build
    if build.needs_build():
        pytest.skip("the library is not built here")
    stamp = open(_lib.LIB_PATH + ".stamp").read()
    assert _lib.REPO_DIR not in stamp and "<repo>" in stamp
    dst = tmp_path / "copy"
    repo = _lib.REPO_DIR
    ignore = shutil.ignore_patterns(".git", "gpurun_out", "*.o", "__pycache__", "profiles", "ab", "variants")
    shutil.copytree(repo, dst, ignore=ignore, symlinks=True)
    code = ("import sys; sys.path.insert(0, %r); from pong_amd import build as B; "
            "print(B.needs_build())" % str(dst / "neuro-genetic-pong-self-play_amd"))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "False"
