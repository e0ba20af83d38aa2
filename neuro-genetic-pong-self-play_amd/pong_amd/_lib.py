"""ctypes binding of ``libpong_ga.so`` (the C-ABI declared in ``include/pong_ga.h``).

The structures below mirror the header field for field.  The library is the
only compute path: if it is missing or cannot be loaded, :func:`lib` raises --
there is no CPU fallback in the product.
"""
from __future__ import annotations

import ctypes
import os
import threading

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_NAME = "libpong_ga.so"
LIB_PATH = os.environ.get("PONG_GA_LIB") or os.path.join(PKG_DIR, LIB_NAME)  # override: variant builds
HEADER_PATH = os.path.join(REPO_DIR, "include", "pong_ga.h")

PG_ABI_VERSION = 12
PG_MAX_NODES = 9

PG_OK, PG_ERR_INVALID, PG_ERR_HIP, PG_ERR_UNSUPPORTED = 0, -1, -2, -3
PG_F32, PG_F64 = 0, 1
PG_OPP_HARDCODED, PG_OPP_ROM_CPU, PG_OPP_SCORE, PG_OPP_NN = 0, 1, 2, 3
PG_PREP_ALL, PG_PREP_GENOMES, PG_PREP_REST = 0, 1, 2
PG_PREC_CERTIFIED, PG_PREC_F64 = 0, 1
PG_SCHED_REFERENCE, PG_SCHED_SELFPLAY = 0, 1
PG_KERNEL_AUTO, PG_KERNEL_GENERAL, PG_KERNEL_RESIDENT, PG_KERNEL_SPLIT, PG_KERNEL_WIDE, PG_KERNEL_STAGED = 0, 1, 2, 3, 4, 5
PG_STATE_FIELDS = 16
STATE_FIELD_NAMES = ("ball_x", "ball_y", "ball_vx", "ball_vy", "ball_visible", "serve_timer",
                     "serve_dir", "hits", "point", "lpy", "rpy", "score1", "score2",
                     "one_player", "seed_lo", "seed_hi")

_vp = ctypes.c_void_p


class PgNet(ctypes.Structure):
    _fields_ = [("n_nodes", ctypes.c_int32), ("nodes", ctypes.c_int32 * PG_MAX_NODES),
                ("bias", ctypes.c_int32), ("dtype", ctypes.c_int32)]


class PgEvalArgs(ctypes.Structure):
    _fields_ = [
        ("struct_size", ctypes.c_uint32),  # ABI 10+: sizeof(pg_eval_args); the library refuses any other value
        ("net", PgNet),
        ("n_genomes", ctypes.c_int32), ("n_games", ctypes.c_int32),
        ("genomes", _vp), ("genome_stride", ctypes.c_int64),
        ("opponents", _vp), ("opponent_stride", ctypes.c_int64), ("n_opponents", ctypes.c_int32),
        ("precision", ctypes.c_int32),
        ("game_kind", _vp), ("game_opp", _vp), ("game_mult", _vp),
        ("seed", ctypes.c_uint64),
        ("fitness", _vp), ("rewards", _vp), ("scores", _vp), ("frames", _vp),
        ("total_frames", _vp), ("status", _vp), ("counters", _vp),
        ("trace", _vp), ("trace_games", ctypes.c_int32), ("trace_cap", ctypes.c_int32),
        ("kernel", ctypes.c_int32), ("group_lanes", ctypes.c_int32),
        ("workspace", _vp), ("workspace_bytes", ctypes.c_size_t),
        ("hard_log", _vp), ("hard_cap", ctypes.c_int32), ("genome_rows", _vp),
        ("n_active", _vp),
        ("prep", ctypes.c_int32), ("horizon", ctypes.c_int32),
        ("timeout_thresh", ctypes.c_int32), ("win_score", ctypes.c_int32),  # ABI 11
    ]

    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        self.struct_size = ctypes.sizeof(PgEvalArgs)


class PgForwardArgs(ctypes.Structure):
    _fields_ = [
        ("net", PgNet), ("n", ctypes.c_int32), ("genomes", _vp), ("genome_stride", ctypes.c_int64),
        ("genome_index", _vp), ("x", _vp), ("precision", ctypes.c_int32), ("index", _vp),
        ("act", _vp), ("counters", _vp), ("z_all", _vp), ("h_all", _vp),
    ]


class PgDecideArgs(ctypes.Structure):
    _fields_ = [
        ("net", PgNet), ("n", ctypes.c_int32), ("genomes", _vp), ("genome_stride", ctypes.c_int64),
        ("genome_index", _vp), ("k", _vp), ("index", _vp), ("stage", _vp),
    ]


class PgWideDecideArgs(ctypes.Structure):
    _fields_ = [
        ("net", PgNet), ("n", ctypes.c_int32), ("genomes", _vp), ("genome_stride", ctypes.c_int64),
        ("genome_index", _vp), ("k", _vp), ("index", _vp), ("act", _vp),
        ("workspace", _vp), ("workspace_bytes", ctypes.c_size_t),
    ]


class PgGaArgs(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int32), ("genes", ctypes.c_int64), ("dtype", ctypes.c_int32),
        ("parents", _vp), ("stride", ctypes.c_int64), ("n_parents", ctypes.c_int32),
        ("chosen", _vp), ("offspring", _vp), ("invalid", _vp),
        ("cxpb", ctypes.c_double), ("mutpb", ctypes.c_double), ("alpha", ctypes.c_double),
        ("mu", ctypes.c_double), ("sigma", ctypes.c_double), ("indpb", ctypes.c_double),
        ("seed", ctypes.c_uint64), ("generation", ctypes.c_uint64), ("pair_mask", _vp),
        ("pair_list", _vp), ("pair_count", _vp), ("pair_cap", ctypes.c_int32),
    ]


class PgSelectArgs(ctypes.Structure):
    _fields_ = [
        ("n_pop", ctypes.c_int32), ("k", ctypes.c_int32), ("tournsize", ctypes.c_int32),
        ("fitness", _vp), ("chosen", _vp), ("seed", ctypes.c_uint64), ("generation", ctypes.c_uint64),
    ]


class PgScheduleArgs(ctypes.Structure):
    _fields_ = [
        ("mode", ctypes.c_int32), ("n", ctypes.c_int32), ("n_games", ctypes.c_int32),
        ("row_offset", ctypes.c_int64), ("n_hof", ctypes.c_int32), ("hof_fitness", _vp),
        ("seed", ctypes.c_uint64), ("generation", ctypes.c_uint64),
        ("kind", _vp), ("opp", _vp), ("mult", _vp), ("rows", _vp),
        ("hof_slices", ctypes.c_int32), ("block_rows", ctypes.c_int32), ("slice_local", ctypes.c_int32),
    ]


class PgHofPackedArgs(ctypes.Structure):
    _fields_ = [("maxsize", ctypes.c_int32), ("hof_n", ctypes.c_int32), ("hof_fitness", _vp), ("k", ctypes.c_int32),
                ("packed", _vp), ("new_n", _vp), ("new_src", _vp), ("new_fitness", _vp),
                ("slot_in", _vp), ("slot_out", _vp)]  # ABI 12: the hall in place


class PgHofArgs(ctypes.Structure):
    _fields_ = [
        ("maxsize", ctypes.c_int32), ("hof_n", ctypes.c_int32), ("hof_fitness", _vp), ("hof_hash", _vp),
        ("pop_n", ctypes.c_int32), ("pop_fitness", _vp), ("pop_hash", _vp), ("rank", _vp),
        ("new_n", _vp), ("new_src", _vp), ("new_fitness", _vp),
    ]


class PgHofRankArgs(ctypes.Structure):
    _fields_ = [
        ("hof_n", ctypes.c_int32), ("hof_fitness", _vp), ("hof_hash", _vp), ("k", ctypes.c_int32),
        ("cand_fitness", _vp), ("cand_hash", _vp), ("packed", _vp), ("workspace", _vp),
        ("workspace_bytes", ctypes.c_size_t),
    ]


class PgHofPrepareArgs(ctypes.Structure):
    _fields_ = [
        ("fitness", _vp), ("pop_n", ctypes.c_int32), ("filter", ctypes.c_int32), ("worst", ctypes.c_double),
        ("rows", _vp), ("stride", ctypes.c_int64), ("genes", ctypes.c_int64), ("dtype", ctypes.c_int32),
        ("hof_n", ctypes.c_int32), ("hof_fitness", _vp), ("hof_hash", _vp), ("k", _vp), ("cand", _vp),
        ("hashes", _vp), ("packed", _vp), ("workspace", _vp), ("workspace_bytes", ctypes.c_size_t),
    ]


class PgScatterArgs(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int32), ("n_games", ctypes.c_int32), ("row_lo", ctypes.c_int32),
        ("fitness", _vp), ("frames", _vp), ("rows", _vp), ("n_active", _vp), ("shard_fitness", _vp),
        ("lineage", _vp),
    ]


class PgMergeArgs(ctypes.Structure):
    _fields_ = [
        ("pop_n", ctypes.c_int32), ("fitness", _vp), ("invalid", _vp), ("inherited", _vp), ("new_fitness", _vp),
        ("filter", ctypes.c_int32), ("worst", ctypes.c_double), ("cand", _vp), ("cand_fitness", _vp),
        ("summary", _vp), ("workspace", _vp), ("workspace_bytes", ctypes.c_size_t),
    ]


class PgHofCandArgs(ctypes.Structure):
    _fields_ = [
        ("hof_n", ctypes.c_int32), ("hof_fitness", _vp), ("hof_hash", _vp), ("k", ctypes.c_int32),
        ("cand", _vp), ("cand_fitness", _vp), ("rows", _vp), ("stride", ctypes.c_int64),
        ("genes", ctypes.c_int64), ("dtype", ctypes.c_int32), ("cand_hash", _vp), ("packed", _vp),
        ("workspace", _vp), ("workspace_bytes", ctypes.c_size_t),
    ]


class PgHofCommitArgs(ctypes.Structure):
    _fields_ = [
        ("dst", _vp), ("dst_stride", ctypes.c_int64), ("old_rows", _vp), ("old_stride", ctypes.c_int64),
        ("rows", _vp), ("rows_stride", ctypes.c_int64), ("cand", _vp), ("src", _vp), ("n_old", ctypes.c_int32),
        ("m", ctypes.c_int32), ("genes", ctypes.c_int64), ("dtype", ctypes.c_int32), ("old_hash", _vp),
        ("cand_hash", _vp), ("new_hash", _vp), ("fitness_in", _vp), ("new_fitness", _vp),
        ("dst_slot", _vp),  # ABI 12: the hall in place
    ]


# name -> (restype, argtypes); exactly the functions include/pong_ga.h declares
SIGNATURES = {
    "pg_version": (ctypes.c_char_p, []),
    "pg_abi_version": (ctypes.c_int32, []),
    "pg_build_flags": (ctypes.c_int32, []),
    "pg_last_error": (ctypes.c_char_p, []),
    "pg_device_count": (ctypes.c_int32, []),
    "pg_eval_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(PgEvalArgs)]),
    "pg_gene_count": (ctypes.c_int32, [ctypes.POINTER(PgNet)]),
    "pg_eval_population": (ctypes.c_int32, [ctypes.POINTER(PgEvalArgs), _vp]),
    "pg_forward": (ctypes.c_int32, [ctypes.POINTER(PgForwardArgs), _vp]),
    "pg_decide": (ctypes.c_int32, [ctypes.POINTER(PgDecideArgs), _vp]),
    "pg_wide_decide_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(PgWideDecideArgs)]),
    "pg_wide_decide": (ctypes.c_int32, [ctypes.POINTER(PgWideDecideArgs), _vp]),
    "pg_physics_reset": (ctypes.c_int32, [_vp, ctypes.c_int32, _vp, _vp, _vp]),
    "pg_physics_step": (ctypes.c_int32, [_vp, ctypes.c_int32, _vp, _vp]),
    "pg_ga_select_tournament": (ctypes.c_int32, [ctypes.POINTER(PgSelectArgs), _vp]),
    "pg_ga_select_tournament_ranked": (ctypes.c_int32, [ctypes.POINTER(PgSelectArgs), _vp, _vp, _vp]),
    "pg_ga_vary": (ctypes.c_int32, [ctypes.POINTER(PgGaArgs), _vp]),
    "pg_ga_list_pairs": (ctypes.c_int32, [_vp, ctypes.c_int32, _vp, _vp, _vp]),
    "pg_ga_mark_pairs": (ctypes.c_int32, [_vp, ctypes.c_int32, _vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                          _vp, _vp]),
    "pg_ga_schedule": (ctypes.c_int32, [ctypes.POINTER(PgScheduleArgs), _vp]),
    "pg_row_hash": (ctypes.c_int32, [_vp, ctypes.c_int64, _vp, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, _vp,
                                     _vp]),
    "pg_hof_update": (ctypes.c_int32, [ctypes.POINTER(PgHofArgs)]),
    "pg_hof_update_packed": (ctypes.c_int32, [ctypes.POINTER(PgHofPackedArgs)]),
    "pg_hof_rank_classes_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int32]),
    "pg_hof_rank_classes": (ctypes.c_int32, [ctypes.POINTER(PgHofRankArgs), _vp]),
    "pg_hof_prepare_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int32, ctypes.c_int32]),
    "pg_hof_prepare": (ctypes.c_int32, [ctypes.POINTER(PgHofPrepareArgs), _vp]),
    "pg_gather_rows": (ctypes.c_int32, [_vp, ctypes.c_int64, _vp, ctypes.c_int64, _vp, ctypes.c_int64, _vp, _vp,
                                        ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, _vp]),
    "pg_ga_scatter_fitness": (ctypes.c_int32, [ctypes.POINTER(PgScatterArgs), _vp]),
    "pg_ga_merge_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int32]),
    "pg_ga_merge_fitness": (ctypes.c_int32, [ctypes.POINTER(PgMergeArgs), _vp]),
    "pg_ga_select_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int32]),
    "pg_ga_select_ranked": (ctypes.c_int32, [ctypes.POINTER(PgSelectArgs), _vp, ctypes.c_size_t, _vp]),
    "pg_ga_inherit": (ctypes.c_int32, [_vp, ctypes.c_int32, _vp, _vp, _vp, _vp, _vp]),
    "pg_ga_order_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int32]),
    "pg_ga_order": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_int32, _vp, _vp, ctypes.c_int32, _vp, _vp, _vp,
                                     ctypes.c_size_t, _vp]),
    "pg_hof_prepare_cand_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int32, ctypes.c_int32]),
    "pg_hof_prepare_cand": (ctypes.c_int32, [ctypes.POINTER(PgHofCandArgs), _vp]),
    "pg_hof_commit": (ctypes.c_int32, [ctypes.POINTER(PgHofCommitArgs), _vp]),
    "pg_render_frames": (ctypes.c_int32, [_vp, ctypes.c_int32, _vp, _vp]),
    "pg_find_stuff": (ctypes.c_int32, [_vp, ctypes.c_int64, ctypes.c_int32, _vp, _vp]),
}

_lock = threading.Lock()
_lib = None


class PongGAError(RuntimeError):
    """A libpong_ga call returned a negative pg_status."""

    def __init__(self, func: str, code: int, message: str):
        super().__init__(f"{func} failed ({code}): {message}")
        self.code = code


def lib() -> ctypes.CDLL:
    """Load libpong_ga.so (built in-tree by ``pong_amd.build``); raise if absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                    "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
            L = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            if L.pg_abi_version() != PG_ABI_VERSION:
                raise RuntimeError(f"{LIB_PATH}: ABI {L.pg_abi_version()} != {PG_ABI_VERSION}")
            _lib = L
    return _lib


def check(func: str, rc: int) -> None:
    if rc != PG_OK:
        msg = lib().pg_last_error()
        raise PongGAError(func, rc, msg.decode() if msg else "")


def make_net(nodes, bias=True, dtype=PG_F64) -> PgNet:
    nodes = [int(n) for n in nodes]
    if not 2 <= len(nodes) <= PG_MAX_NODES:
        raise ValueError(f"NETWORK_SHAPE must have 2..{PG_MAX_NODES} entries, got {nodes}")
    arr = (ctypes.c_int32 * PG_MAX_NODES)(*(nodes + [0] * (PG_MAX_NODES - len(nodes))))
    return PgNet(len(nodes), arr, 1 if bias else 0, dtype)
