"""ctypes wrapper of the CPU oracle (``oracle/pong_oracle.c``).

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker or the timed CPU baseline -- never as the thing measured or shipped.
The product path (``neuro-genetic-pong-self-play_amd/``) never imports it.

What it restates (reference file:line) is listed in ``pong_oracle.h``.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

OPP_HARDCODED, OPP_ROM_CPU, OPP_SCORE, OPP_NN = 0, 1, 2, 3

_lib = None


def build(force: bool = False) -> str:
    """Compile the oracle with its Makefile (gcc); returns the .so path."""
    src = os.path.join(HERE, "pong_oracle.c")
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


class OrState(ctypes.Structure):
    _fields_ = [
        ("ball_x", ctypes.c_int), ("ball_y", ctypes.c_int),
        ("ball_vx", ctypes.c_int), ("ball_vy", ctypes.c_int),
        ("ball_visible", ctypes.c_int), ("serve_timer", ctypes.c_int),
        ("serve_dir", ctypes.c_int), ("hits", ctypes.c_int), ("point", ctypes.c_int),
        ("lpy", ctypes.c_int), ("rpy", ctypes.c_int),
        ("score1", ctypes.c_int), ("score2", ctypes.c_int),
        ("one_player", ctypes.c_int),
        ("seed", ctypes.c_uint64),
    ]


class OrNet(ctypes.Structure):
    _fields_ = [("n_nodes", ctypes.c_int), ("nodes", ctypes.POINTER(ctypes.c_int)),
                ("bias", ctypes.c_int)]


class OrGameResult(ctypes.Structure):
    _fields_ = [("score1", ctypes.c_int), ("score2", ctypes.c_int), ("frames", ctypes.c_int),
                ("total_frames", ctypes.c_double), ("reward", ctypes.c_double),
                ("zero_division", ctypes.c_int), ("slow_decisions", ctypes.c_int)]


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int32)
        L.or_splitmix64.restype = ctypes.c_uint64
        L.or_splitmix64.argtypes = [ctypes.c_uint64]
        L.or_game_seed.restype = ctypes.c_uint64
        L.or_game_seed.argtypes = [ctypes.c_uint64, ctypes.c_int]
        L.or_env_reset.argtypes = [ctypes.POINTER(OrState), ctypes.c_uint64, ctypes.c_int]
        L.or_env_step.argtypes = [ctypes.POINTER(OrState)] + [ctypes.c_int] * 4
        L.or_env_done.argtypes = [ctypes.POINTER(OrState)]
        L.or_gene_count.argtypes = [ctypes.POINTER(OrNet)]
        L.or_nn_run.argtypes = [dp, ctypes.POINTER(OrNet), dp, dp]
        L.or_blas_gemv.argtypes = [dp, ctypes.c_int, ctypes.c_int, dp, dp]
        L.or_blas_gemv.restype = None
        L.or_play_game.argtypes = [dp, ctypes.POINTER(OrNet), ctypes.c_int, dp, ctypes.c_double,
                                   ctypes.c_uint64, ctypes.POINTER(OrGameResult),
                                   ctypes.POINTER(ctypes.c_uint8), ctypes.c_int]
        L.or_play_slot.argtypes = [dp, ctypes.POINTER(OrNet), ctypes.c_int, dp, ctypes.c_double,
                                   ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(OrGameResult),
                                   ctypes.POINTER(ctypes.c_uint8), ctypes.c_int]
        L.or_eval_population_h.restype = ctypes.c_int
        L.or_eval_population_h.argtypes = [
            ctypes.c_int, ctypes.c_int, dp, ctypes.c_int64, dp, ctypes.c_int64, ip, ip, dp,
            ctypes.POINTER(OrNet), ctypes.c_uint64, ctypes.c_int, dp, dp, ip, ip, dp, ip, ctypes.c_int]
        L.or_eval_population.restype = ctypes.c_int
        L.or_eval_population.argtypes = [
            ctypes.c_int, ctypes.c_int, dp, ctypes.c_int64, dp, ctypes.c_int64, ip, ip, dp,
            ctypes.POINTER(OrNet), ctypes.c_uint64, dp, dp, ip, ip, dp, ip, ctypes.c_int]
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.or_render.argtypes = [ctypes.POINTER(OrState), u8p]
        L.or_find_stuff.argtypes = [u8p, dp]
        L.or_set_limits.argtypes = [ctypes.c_int, ctypes.c_int]
        L.or_set_limits.restype = None
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)) if a is not None else None


def _ip(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)) if a is not None else None


class Net:
    """Keeps the ctypes network descriptor and its node array alive."""

    def __init__(self, nodes, bias=True):
        self.nodes_arr = (ctypes.c_int * len(nodes))(*[int(n) for n in nodes])
        self.s = OrNet(len(nodes), self.nodes_arr, 1 if bias else 0)
        self.nodes = list(nodes)
        self.bias = bool(bias)

    @property
    def ref(self):
        return ctypes.byref(self.s)

    def gene_count(self) -> int:
        return lib().or_gene_count(self.ref)


def splitmix64(x: int) -> int:
    return lib().or_splitmix64(x)


def game_seed(base_seed: int, game_index: int) -> int:
    return lib().or_game_seed(base_seed, game_index)


def nn_run(genes, nodes, x, bias=True):
    """numpy_nn.NeuralNetwork.run restated: returns (argmax index, final activations)."""
    net = Net(nodes, bias)
    g = np.ascontiguousarray(genes, dtype=np.float64)
    xx = np.ascontiguousarray(x, dtype=np.float64)
    out = np.zeros(nodes[-1], dtype=np.float64)
    idx = lib().or_nn_run(_dp(g), net.ref, _dp(xx), _dp(out))
    return idx, out


def blas_gemv(w, x):
    """np.dot(w, x) restated in OpenBLAS dgemv_t's operation order (pong_oracle.c or_blas_dot)."""
    w = np.ascontiguousarray(w, dtype=np.float64)
    xx = np.ascontiguousarray(x, dtype=np.float64)
    n, m = w.shape
    assert xx.shape == (m,)
    y = np.zeros(n, dtype=np.float64)
    lib().or_blas_gemv(_dp(w), n, m, _dp(xx), _dp(y))
    return y


class Env:
    """The oracle physics behind the reference's env interface (step/reset/close)."""

    def __init__(self, seed: int, one_player: bool = False):
        self.state = OrState()
        self.seed = seed
        self.one_player = one_player
        lib().or_env_reset(ctypes.byref(self.state), seed, int(one_player))

    def reset(self):
        lib().or_env_reset(ctypes.byref(self.state), self.seed, int(self.one_player))

    def step4(self, r_up, r_dn, l_up, l_dn):
        lib().or_env_step(ctypes.byref(self.state), int(r_up), int(r_dn), int(l_up), int(l_dn))

    def done(self) -> bool:
        return bool(lib().or_env_done(ctypes.byref(self.state)))

    def snapshot(self) -> dict:
        return {name: getattr(self.state, name) for name, _ in OrState._fields_}


class limits:
    """Context manager: the episode limits (or_set_limits; TIMEOUT_THRESH and
    WIN_SCORE of config.py, pg_eval_args.timeout_thresh / win_score) for the
    calls inside it; 0 = the reference's 2000 / 3."""

    def __init__(self, timeout_thresh=0, win_score=0):
        self.t, self.w = int(timeout_thresh), int(win_score)

    def __enter__(self):
        lib().or_set_limits(self.t, self.w)
        return self

    def __exit__(self, *exc):
        lib().or_set_limits(0, 0)
        return False


def play_game(genes, nodes, opp_kind, opp_genes=None, mult=1.0, seed=0, bias=True, trace_cap=0, horizon=0,
              timeout_thresh=0, win_score=0):
    """One game slot (or_play_slot): a perform_episode, or with ``horizon`` > 0
    the fixed-horizon mode (T frames, auto-reset; pong_ga.h pg_eval_args.horizon)."""
    with limits(timeout_thresh, win_score):
        return _play_game(genes, nodes, opp_kind, opp_genes, mult, seed, bias, trace_cap, horizon)


def _play_game(genes, nodes, opp_kind, opp_genes, mult, seed, bias, trace_cap, horizon):
    net = Net(nodes, bias)
    g = np.ascontiguousarray(genes, dtype=np.float64)
    og = np.ascontiguousarray(opp_genes, dtype=np.float64) if opp_genes is not None else None
    res = OrGameResult()
    trace = (ctypes.c_uint8 * max(trace_cap, 1))()
    lib().or_play_slot(_dp(g), net.ref, int(opp_kind), _dp(og), float(mult), seed, int(horizon),
                       ctypes.byref(res), trace if trace_cap else None, int(trace_cap))
    out = {k: getattr(res, k) for k, _ in OrGameResult._fields_}
    if trace_cap:
        out["trace"] = np.frombuffer(bytes(trace), dtype=np.uint8)[: min(res.frames, trace_cap)].copy()
    return out


def eval_population(genomes, nodes, kind, opp_index, mult, opponents=None, bias=True,
                    base_seed=0, n_threads=0, horizon=0, timeout_thresh=0, win_score=0):
    """Whole-population evaluate(): returns a dict of numpy arrays (``horizon`` > 0:
    every game slot in the fixed-horizon mode, or_eval_population_h; ``timeout_thresh``,
    ``win_score``: config.py's TIMEOUT_THRESH / WIN_SCORE, 0 = the reference's)."""
    with limits(timeout_thresh, win_score):
        return _eval_population(genomes, nodes, kind, opp_index, mult, opponents, bias, base_seed, n_threads,
                                horizon)


def _eval_population(genomes, nodes, kind, opp_index, mult, opponents, bias, base_seed, n_threads, horizon):
    net = Net(nodes, bias)
    G = np.ascontiguousarray(genomes, dtype=np.float64)
    n = G.shape[0]
    kind = np.ascontiguousarray(kind, dtype=np.int32)
    n_games = kind.shape[1] if kind.ndim == 2 else 6
    opp_index = np.ascontiguousarray(opp_index, dtype=np.int32)
    mult = np.ascontiguousarray(mult, dtype=np.float64)
    if opponents is None:
        opponents = np.zeros((1, G.shape[1] if G.ndim == 2 else 1), dtype=np.float64)
    O = np.ascontiguousarray(opponents, dtype=np.float64)
    fitness = np.zeros(n, np.float64)
    rewards = np.zeros((n, n_games), np.float64)
    scores = np.zeros((n, n_games, 2), np.int32)
    frames = np.zeros((n, n_games), np.int32)
    total = np.zeros((n, n_games), np.float64)
    status = np.zeros(n, np.int32)
    first_err = lib().or_eval_population_h(
        n, n_games, _dp(G), G.shape[1] if n else 0, _dp(O), O.shape[1], _ip(kind), _ip(opp_index),
        _dp(mult), net.ref, base_seed, int(horizon), _dp(fitness), _dp(rewards), _ip(scores), _ip(frames),
        _dp(total), _ip(status), int(n_threads))
    return {"fitness": fitness, "rewards": rewards, "scores": scores, "frames": frames,
            "total_frames": total, "status": status, "first_error": first_err}


# ------------------------------------------------------------- pixel path
def render(state: dict) -> np.ndarray:
    """or_render: the [210, 160, 3] uint8 frame of a state (Env.snapshot() keys)."""
    s = OrState(**{k: int(state[k]) for k in ("ball_x", "ball_y", "ball_visible", "lpy", "rpy")})
    frame = np.zeros((210, 160, 3), dtype=np.uint8)
    lib().or_render(ctypes.byref(s), frame.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    return frame


def find_stuff(frame: np.ndarray) -> np.ndarray:
    """or_find_stuff: [3, 2] f64 centroids (ball, left, right), NaN for None."""
    f = np.ascontiguousarray(frame, dtype=np.uint8)
    if f.shape != (210, 160, 3):
        raise ValueError("frame must be [210, 160, 3] uint8")
    out = np.zeros(6, dtype=np.float64)
    lib().or_find_stuff(f.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), _dp(out))
    return out.reshape(3, 2)
