#!/usr/bin/env python3
"""Generate the golden vectors from the REAL reference code.

Runs only in the build container, where the read-only reference lives at
/root/reference.  It imports the reference's policy-side modules
(numpy_nn.py, utils.py, dumb_ais.py, config.py) and AST-extracts the episode
functions of main.py (perform_episode, get_actions,
calculate_timeout_and_frames, evaluate), then runs them and writes the
inputs/outputs as small fixtures next to this script.  The fixtures are data;
no reference source travels with them.

Shims (all documented in DESIGN.md "Oracle"):
  * ``np.int = int``: config.py:21,26 use ``np.int`` (removed in numpy 1.24).
  * a stub ``scoop`` module with only ``logger`` (numpy_nn.py:67, utils.py:160).
  * ``find_stuff`` with the ball absent but paddles present: numpy >= 1.24
    refuses the ragged ``np.array([None, arr, arr])`` (utils.py:19); the shim
    catches that ValueError and builds the same 3-element object array numpy
    < 1.24 returned, from the reference's own ``get_rect_quickly``.
  * ``NeuralNetwork.run`` for 3-output networks raises on argmax index 2
    (numpy_nn.py:136-137); the build maps index 2 to ``[0, 0]`` (no-op), and
    the shim does the same so whole-episode traces can be recorded.
  * ``retro``: absent (third-party emulator).  A fake env steps the build's
    physics through the CPU oracle (oracle/liboracle.so) and renders
    210x160x3 frames in the config.py colours, so the reference's pixel path
    (find_stuff) reads the positions exactly as it would read the emulator's.
  * the hall of fame is a stub with DEAP's ``items`` list and
    ``fitness.valid/values`` (deap is absent).

Usage:  python tests/golden/make_golden.py   (takes a few minutes)
        python tests/golden/make_golden.py episodes_s3 wide_s3 evaluate_s3   (round-2 additions)
        python tests/golden/make_golden.py hard_cases gpurun_out/.../hard_cases.npz
        (nn_hard_cases.npz from a tools/harvest_hard.py run on the GPU)
"""
from __future__ import annotations

import ast
import hashlib
import json
import logging
import os
import random
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as O  # noqa: E402  (the build's physics, for the fake env)

# ---------------------------------------------------------------- shims ----
np.int = int  # type: ignore[attr-defined]
_scoop = types.ModuleType("scoop")
_scoop.logger = logging.getLogger("scoop-stub")
sys.modules["scoop"] = _scoop
sys.path.insert(0, REF)

import config as ref_config  # noqa: E402
import dumb_ais as ref_dumb  # noqa: E402
import numpy_nn as ref_nn  # noqa: E402
import utils as ref_utils  # noqa: E402

_orig_find_stuff = ref_utils.find_stuff


def _find_stuff_np1(observation):
    try:
        return _orig_find_stuff(observation)
    except ValueError:
        chopped = observation[ref_config.GAME_TOP:ref_config.GAME_BOTTOM, :]
        out = np.empty(3, dtype=object)
        out[:] = [ref_utils.get_rect_quickly(chopped, c) for c in
                  (ref_config.BALL_COLOUR, ref_config.LEFT_GUY_COLOUR, ref_config.RIGHT_GUY_COLOUR)]
        return out


_orig_run = ref_nn.NeuralNetwork.run


def _run_noop_on_index2(self, input_vector):
    try:
        return _orig_run(self, input_vector)
    except Exception as e:  # "Shouldn't happen": argmax index >= 2
        if str(e) != "Shouldn't happen":
            raise
        return [0, 0]


ref_nn.NeuralNetwork.run = _run_noop_on_index2


def extract_main_functions(names):
    src = open(os.path.join(REF, "main.py")).read()
    tree = ast.parse(src)
    keep = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in names]
    return ast.Module(body=keep, type_ignores=[])


# ------------------------------------------------------------- fake env ----
def render(state: dict) -> np.ndarray:
    """210x160x3 frame of the oracle state in the reference colours (obs.npy layout)."""
    f = np.empty((210, 160, 3), dtype=np.uint8)
    f[:] = ref_config.BG_COLOUR
    f[24:34] = ref_config.BALL_COLOUR      # top wall (outside the crop)
    f[194:210] = ref_config.BALL_COLOUR    # bottom wall (outside the crop)
    top = ref_config.GAME_TOP
    for py, x0, col in ((state["lpy"], 16, ref_config.LEFT_GUY_COLOUR),
                        (state["rpy"], 140, ref_config.RIGHT_GUY_COLOUR)):
        lo, hi = max(py, 0), min(py + 15, 159)
        f[top + lo: top + hi + 1, x0:x0 + 4] = col
    if state["ball_visible"]:
        by, bx = state["ball_y"], state["ball_x"]
        f[top + by: top + by + 4, bx:bx + 2] = ref_config.BALL_COLOUR
    return f


class FakeEnv:
    def __init__(self, game_index: int, one_player: bool):
        self.env = O.Env(O.game_seed(0, game_index), one_player)
        self.use_restricted_actions = None
        self.received = []
        self.last_info = {"score1": 0, "score2": 0}

    def reset(self):
        self.env.reset()
        return render(self.env.snapshot())

    def step(self, action):
        a = [int(v) for v in action]
        self.received.append(a)
        self.env.step4(a[4], a[5], a[6], a[7])
        s = self.env.snapshot()
        info = {"score1": s["score1"], "score2": s["score2"]}
        self.last_info = dict(info)
        return render(s), 0.0, self.env.done(), info

    def close(self):
        pass


class FakeRetro(types.ModuleType):
    """`retro.make` stand-in: evaluate() makes one env per game, in order."""

    class Actions:
        FILTERED = "FILTERED"

    def __init__(self):
        super().__init__("retro")
        self.calls = 0
        self.envs = []

    def make(self, game, state=None, players=1):
        env = FakeEnv(self.calls % ref_config.GAMES_TO_PLAY, one_player=(state is None))
        self.calls += 1
        self.envs.append(env)
        return env


# ------------------------------------------------------------ HoF stub -----
class _Fit:
    def __init__(self, value):
        self.values = (value,)
        self.valid = True


class _Ind(list):
    def __init__(self, genes, fitness):
        super().__init__(genes)
        self.fitness = _Fit(fitness)


class _HoF:
    def __init__(self, items):
        self.items = items


def make_namespace(network_shape, hall_of_fame=None):
    ns = {}
    ns.update({k: getattr(ref_utils, k) for k in dir(ref_utils) if not k.startswith("__")})
    ref_utils.NETWORK_SHAPE = list(network_shape)
    ns["NETWORK_SHAPE"] = list(network_shape)
    ns["find_stuff"] = _find_stuff_np1
    ns["HardcodedAi"] = ref_dumb.HardcodedAi
    ns["ScoreHardcodedAi"] = ref_dumb.ScoreHardcodedAi
    ns["time"] = __import__("time")
    ns["np"] = np
    ns["retro"] = FakeRetro()
    ns["hall_of_fame"] = hall_of_fame
    ns["RENDER"] = False
    code = compile(extract_main_functions(
        {"perform_episode", "get_actions", "calculate_timeout_and_frames", "evaluate"}),
        os.path.join(REF, "main.py"), "exec")
    exec(code, ns)
    return ns


# --------------------------------------------------------------- helpers ---
def f32(a):
    return np.asarray(a, dtype=np.float32).astype(np.float64)


def gene_count(shape, bias=True):
    b = 1 if bias else 0
    return sum((shape[i] + b) * shape[i + 1] for i in range(len(shape) - 1))


def gen_genes(rng, dist, g):
    if dist == "init":
        return f32(rng.random(g))
    sigma = float(dist[1:])
    return f32(rng.standard_normal(g) * sigma)


DISTS = ["init", "n1", "n3", "n9", "n30"]


def gen_nn_forward():
    rng = np.random.default_rng(20240601)
    out = {}
    cases = [([6, 2, 2], True, 8, 32), ([6, 64, 2], True, 6, 32), ([6, 64, 3], True, 8, 48),
             ([6, 8, 8, 3], True, 6, 32), ([6, 4, 2], False, 6, 32)]
    for shape, bias, n_genomes, n_inputs in cases:
        key = "x".join(map(str, shape)) + ("" if bias else "_nobias")
        G = gene_count(shape, bias)
        genes, gidx, xs, acts, idxs = [], [], [], [], []
        for dist in DISTS:
            for _ in range(n_genomes):
                g = gen_genes(rng, dist, G)
                genes.append(g)
                net = ref_nn.NeuralNetwork(nodes=list(shape), weights=list(g), bias=bias)
                for k in range(n_inputs):
                    if k % 2 == 0:  # the game's exact k/320 features
                        x = rng.integers(0, 321, size=6) / 320.0
                    else:
                        x = rng.random(6)
                    x = [float(v) for v in x]
                    try:
                        net.run(x)
                    except Exception:
                        pass
                    last = net.list_of_transitional_arrays[-1]
                    a = np.array(last[:-1] if bias else last, dtype=np.float64)
                    gidx.append(len(genes) - 1)
                    xs.append(x)
                    acts.append(a)
                    idxs.append(int(np.argmax(a)))
        out[key] = dict(shape=np.array(shape), bias=np.array(bias), genes=np.array(genes),
                        gidx=np.array(gidx), x=np.array(xs), act=np.array(acts), idx=np.array(idxs))
    np.savez_compressed(os.path.join(HERE, "nn_forward.npz"),
                        **{f"{k}__{f}": v for k, d in out.items() for f, v in d.items()})
    # the wide net: genes from a seeded generator (checksum recorded), 4 inputs
    shape = [6, 512, 512, 3]
    G = gene_count(shape)
    wide = []
    for seed, sigma in ((7, 0.05), (8, 1.0)):
        g = f32(np.random.default_rng(seed).standard_normal(G) * sigma)
        net = ref_nn.NeuralNetwork(nodes=shape, weights=list(g), bias=True)
        xr = np.random.default_rng(seed + 100)
        for _ in range(4):
            x = [float(v) for v in xr.integers(0, 321, size=6) / 320.0]
            try:
                net.run(x)
            except Exception:
                pass
            a = np.array(net.list_of_transitional_arrays[-1][:-1], dtype=np.float64)
            wide.append(dict(seed=seed, sigma=sigma, x=x, act=a.tolist(), idx=int(np.argmax(a)),
                             genes_sha256=hashlib.sha256(g.tobytes()).hexdigest()))
    with open(os.path.join(HERE, "nn_forward_wide.json"), "w") as fh:
        json.dump(wide, fh, indent=1)


class _Recorder:
    def __init__(self):
        self.seen = None

    def run(self, x):
        self.seen = [float(v) for v in x]
        return [1, 0]


def gen_helpers():
    rng = np.random.default_rng(99)
    h = {}
    # inference (utils.py:139-153): ball/last/me/enemy are (row, col) centroids
    inf = []
    for _ in range(200):
        ball = [float(rng.integers(0, 320)) / 2, float(rng.integers(0, 320)) / 2]
        last = [float(rng.integers(0, 320)) / 2, float(rng.integers(0, 320)) / 2]
        me = [float(rng.integers(0, 320)) / 2, 141.5]
        enemy = [float(rng.integers(0, 320)) / 2, 17.5]
        rec = _Recorder()
        ref_utils.inference(ball, last, me, enemy, rec)
        inf.append(dict(ball=ball, last=last, me=me, enemy=enemy, features=rec.seen))
    h["inference"] = inf
    # keep_within_game_bounds_please (utils.py:71-77)
    clamp = []
    for y in (0.0, 3.5, 15.0, 15.5, 16.0, 16.5, 80.0, 143.5, 144.0, 144.5, 150.0, 159.0):
        for a in ([0, 0], [1, 0], [0, 1]):
            clamp.append(dict(paddle=[y, 17.5], action=a,
                              out=list(ref_utils.keep_within_game_bounds_please(np.array([y, 17.5]), a))))
    clamp.append(dict(paddle=None, action=[1, 0], out=list(ref_utils.keep_within_game_bounds_please(None, [1, 0]))))
    h["clamp"] = clamp
    # calculate_reward (utils.py:104-109)
    rew = []
    for mult in (1, 1.0, 0.5, -0.75, 2.3125, 0.1, -3.0):
        for total in (1.0, 7.0, 100.0, 333.0, 2047.0, 4095.0):
            for my, en in ((3, 0), (0, 3), (3, 2), (1, 0), (2, 3), (1, 2)):
                rew.append(dict(mult=mult, total=total, my=my, enemy=en,
                                reward=ref_utils.calculate_reward(mult, total, my, en)))
    h["reward"] = rew
    # calculate_timeout_and_frames (main.py:128-135) over score sequences
    ns = make_namespace([6, 2, 2])
    tof = []
    for _ in range(20):
        seq = []
        s1 = s2 = 0
        for _ in range(int(rng.integers(5, 60))):
            r = rng.random()
            if r < 0.08:
                s1 += 1
            elif r < 0.16:
                s2 += 1
            seq.append({"score1": s1, "score2": s2})
        last, t, tot = None, 0.0, 0.0
        steps = []
        for info in seq:
            t, tot = ns["calculate_timeout_and_frames"](last, info, t, tot)
            last = info
            steps.append([t, tot])
        tof.append(dict(seq=[[d["score1"], d["score2"]] for d in seq], out=steps))
    h["timeout_frames"] = tof
    # dumb AIs (dumb_ais.py)
    ais = []
    for _ in range(100):
        x = [float(v) for v in rng.integers(0, 321, size=6) / 320.0]
        if rng.random() < 0.2:
            x[4] = x[1]
        s1, s2 = int(rng.integers(0, 3)), int(rng.integers(0, 3))
        sc = ref_dumb.ScoreHardcodedAi()
        sc.set_score({"score1": s1, "score2": s2})
        ais.append(dict(x=x, score=[s1, s2], hard=ref_dumb.HardcodedAi().run(x), score_ai=sc.run(x)))
    h["dumb_ais"] = ais
    # calculate_gene_size (utils.py:128-136)
    sizes = []
    for shape in ([6, 2, 2], [6, 64, 2], [6, 64, 3], [6, 512, 512, 3], [6, 8, 8, 3]):
        ref_utils.NETWORK_SHAPE = shape
        sizes.append(dict(shape=shape, genes=ref_utils.calculate_gene_size()))
    ref_utils.NETWORK_SHAPE = ref_config.NETWORK_SHAPE
    h["gene_size"] = sizes
    # get_actions (main.py:138-154) with the ball hidden or shown (paddles shown)
    ga = []
    for _ in range(60):
        ball = None if rng.random() < 0.3 else np.array([float(rng.integers(0, 320)) / 2, float(rng.integers(40, 280)) / 2])
        lastb = None if rng.random() < 0.3 else np.array([float(rng.integers(0, 320)) / 2, float(rng.integers(40, 280)) / 2])
        left = np.array([float(rng.integers(0, 320)) / 2, 17.5])
        right = np.array([float(rng.integers(0, 320)) / 2, 141.5])
        la, ra = ns["get_actions"](ball, lastb, left, ref_dumb.HardcodedAi(), right, ref_dumb.HardcodedAi())
        ga.append(dict(ball=None if ball is None else ball.tolist(),
                       last=None if lastb is None else lastb.tolist(),
                       left=left.tolist(), right=right.tolist(), left_action=list(map(int, la)),
                       right_action=list(map(int, ra))))
    h["get_actions"] = ga
    # the reference's own test fixture: find_stuff on obs.npy and a zero frame (tests.py:48-57)
    obs = np.load(os.path.join(REF, "obs.npy"))
    fs = _find_stuff_np1(obs)
    h["find_stuff_obs"] = [list(map(float, v)) for v in fs]
    h["find_stuff_zero"] = [None if v is None else list(map(float, v)) for v in _find_stuff_np1(np.zeros_like(obs))]
    # config.py surface: every upper-case name and its value
    cfg = {}
    for name in dir(ref_config):
        if name.isupper():
            v = getattr(ref_config, name)
            cfg[name] = v.tolist() if isinstance(v, np.ndarray) else (list(v) if isinstance(v, tuple) else v)
    h["config"] = cfg
    with open(os.path.join(HERE, "helpers.json"), "w") as fh:
        json.dump(h, fh, indent=0)


def gen_centroids():
    """find_stuff on frames rendered from physics states: pins the analytic centroids."""
    rng = np.random.default_rng(5)
    rows = []
    for _ in range(300):
        st = dict(lpy=int(rng.integers(-8, 153)), rpy=int(rng.integers(-8, 153)),
                  ball_visible=int(rng.random() < 0.8), ball_y=int(rng.integers(0, 157)),
                  ball_x=int(rng.integers(20, 139)))
        fs = _find_stuff_np1(render(st))
        rows.append([st["lpy"], st["rpy"], st["ball_visible"], st["ball_y"], st["ball_x"]] +
                    ([-1.0, -1.0] if fs[0] is None else list(map(float, fs[0]))) +
                    list(map(float, fs[1])) + list(map(float, fs[2])))
    np.save(os.path.join(HERE, "centroids.npy"), np.array(rows, dtype=np.float64))


def gen_episodes():
    """perform_episode traces: the actions each env.step received, scores, reward."""
    rng = np.random.default_rng(31)
    eps = []
    cases = []
    for shape in ([6, 2, 2], [6, 64, 3]):
        G = gene_count(shape)
        for dist in ("init", "n1", "n3", "n30"):
            right = gen_genes(rng, dist, G)
            opp = gen_genes(rng, dist, G)
            for kind in (O.OPP_HARDCODED, O.OPP_ROM_CPU, O.OPP_SCORE, O.OPP_NN):
                cases.append((shape, dist, kind, right, opp))
    for shape, dist, kind, right, opp in cases:
        ns = make_namespace(shape)
        game_index = {O.OPP_HARDCODED: 0, O.OPP_ROM_CPU: 1, O.OPP_SCORE: 2, O.OPP_NN: 3}[kind]
        env = FakeEnv(game_index, one_player=(kind == O.OPP_ROM_CPU))
        right_model = ref_utils.create_model_from_genes(list(right))
        if kind == O.OPP_NN:
            left_model = ref_utils.create_model_from_genes(list(opp))
        elif kind == O.OPP_SCORE:
            left_model = ref_dumb.ScoreHardcodedAi()
        else:
            left_model = ref_dumb.HardcodedAi()
        mult = 1 if kind != O.OPP_NN else float(np.round(rng.normal(), 3))
        env.reset()
        reward = ns["perform_episode"](env, left_model, right_model, False, mult)
        rec = np.array(env.received, dtype=np.int64)
        st = env.last_info  # perform_episode resets the env on exit (main.py:108)
        eps.append(dict(shape=shape, dist=dist, kind=kind, game_index=game_index, mult=mult,
                        right=right.tolist(), opp=opp.tolist() if kind == O.OPP_NN else None,
                        right_actions=(rec[:, 4] + 2 * rec[:, 5]).tolist(),
                        left_actions=(rec[:, 6] + 2 * rec[:, 7]).tolist(),
                        frames=len(env.received), score1=st["score1"], score2=st["score2"],
                        reward=float(reward)))
        print(f"episode {shape} {dist} kind={kind}: frames={len(env.received)} "
              f"score={st['score1']}-{st['score2']} reward={reward}", flush=True)
    with open(os.path.join(HERE, "episodes.json"), "w") as fh:
        json.dump(eps, fh)


def gen_episodes_s3():
    """More perform_episode traces at the bench's gene scale ([6,64,3], N(0, 3)):
    every game slot of evaluate() (0 HardcodedAi, 1 the ROM CPU, 2
    ScoreHardcodedAi, 3-5 network opponents with negative and fractional
    right_score_multiplier), long rallies, and games that end at the
    2 000-frame timeout -- the periodic rallies the kernels jump over when
    not tracing.  Candidates are screened with the CPU oracle (the build's
    physics) and then played by the REAL perform_episode."""
    rng = np.random.default_rng(303)
    shape = [6, 64, 3]
    G = gene_count(shape)
    kinds = [O.OPP_HARDCODED, O.OPP_ROM_CPU, O.OPP_SCORE, O.OPP_NN, O.OPP_NN, O.OPP_NN]
    picked = []  # (slot, right, opp, mult, tag)
    # quotas: 2 games per slot; 6 timeouts and 6 long rallies (500-2000
    # frames), at least 3 of each against a network opponent; no two picks
    # with the same slot, frames and score (N(0, 3) networks often saturate to
    # one action and replay the same game)
    quota = {"slot": [2] * 6, "timeout": 6, "long": 6, "timeout_nn": 3, "long_nn": 3}
    seen = set()
    tries = 0
    while tries < 20000 and (max(quota["slot"]) > 0 or quota["timeout"] > 0 or quota["long"] > 0):
        tries += 1
        slot = tries % 6
        right = rng.standard_normal(G) * 3.0
        opp = rng.standard_normal(G) * 3.0
        mult = float(np.round(rng.uniform(-1.5, 1.0), 3)) if kinds[slot] == O.OPP_NN else 1.0
        r = O.play_game(right, shape, kinds[slot], opp if kinds[slot] == O.OPP_NN else None, mult,
                        seed=O.game_seed(0, slot))
        sig = (slot, r["frames"], r["score1"], r["score2"])
        if sig in seen:
            continue
        nn = kinds[slot] == O.OPP_NN
        tag = None
        for t, ok in (("timeout", r["frames"] > 2000), ("long", 500 <= r["frames"] <= 2000)):
            # keep room for the network-opponent share of each quota
            if ok and quota[t] > 0 and (nn or quota[t] > quota[t + "_nn"]):
                tag = t
                quota[t] -= 1
                if nn:
                    quota[t + "_nn"] = max(0, quota[t + "_nn"] - 1)
                break
        if tag is None and quota["slot"][slot] > 0:
            tag = "slot"
            quota["slot"][slot] -= 1
        if tag is None:
            continue
        seen.add(sig)
        picked.append((slot, right, opp, mult, tag))
    eps = []
    for slot, right, opp, mult, tag in picked:
        ns = make_namespace(shape)
        kind = kinds[slot]
        env = FakeEnv(slot, one_player=(kind == O.OPP_ROM_CPU))
        right_model = ref_utils.create_model_from_genes(list(right))
        if kind == O.OPP_NN:
            left_model = ref_utils.create_model_from_genes(list(opp))
        elif kind == O.OPP_SCORE:
            left_model = ref_dumb.ScoreHardcodedAi()
        else:
            left_model = ref_dumb.HardcodedAi()
        env.reset()
        reward = ns["perform_episode"](env, left_model, right_model, False, mult)
        rec = np.array(env.received, dtype=np.int64)
        st = env.last_info
        eps.append(dict(shape=shape, dist="n3", kind=kind, game_index=slot, mult=mult, tag=tag,
                        right=right.tolist(), opp=opp.tolist() if kind == O.OPP_NN else None,
                        right_actions=(rec[:, 4] + 2 * rec[:, 5]).tolist(),
                        left_actions=(rec[:, 6] + 2 * rec[:, 7]).tolist(),
                        frames=len(env.received), score1=st["score1"], score2=st["score2"],
                        reward=float(reward)))
        print(f"episode s3 slot={slot} {tag}: frames={len(env.received)} "
              f"score={st['score1']}-{st['score2']} reward={reward}", flush=True)
    with open(os.path.join(HERE, "episodes_s3.json"), "w") as fh:
        json.dump(eps, fh)


def gen_wide_s3():
    """NeuralNetwork.run of the wide net at the wide bench's gene scale (N(0, 3)),
    16 inputs each on the game's k/320 grid, seeds 9 and 10."""
    shape = [6, 512, 512, 3]
    G = gene_count(shape)
    wide = []
    for seed in (9, 10):
        g = f32(np.random.default_rng(seed).standard_normal(G) * 3.0)
        net = ref_nn.NeuralNetwork(nodes=shape, weights=list(g), bias=True)
        xr = np.random.default_rng(seed + 100)
        for _ in range(16):
            x = [float(v) for v in xr.integers(0, 321, size=6) / 320.0]
            try:
                net.run(x)
            except Exception:
                pass
            a = np.array(net.list_of_transitional_arrays[-1][:-1], dtype=np.float64)
            wide.append(dict(seed=seed, sigma=3.0, x=x, act=a.tolist(), idx=int(np.argmax(a)),
                             genes_sha256=hashlib.sha256(g.tobytes()).hexdigest()))
    with open(os.path.join(HERE, "nn_forward_wide_s3.json"), "w") as fh:
        json.dump(wide, fh, indent=1)


def gen_evaluate_s3():
    """Whole evaluate() calls at the bench's gene scale: 6 [6,64,3] individuals
    with N(0, 3) genes against a 5-member N(0, 3) hall of fame whose fitness
    values include negative ones (right_score_multiplier < 0)."""
    rng = np.random.default_rng(707)
    shape, G = [6, 64, 3], gene_count([6, 64, 3])
    inds = [rng.standard_normal(G) * 3.0 for _ in range(6)]
    hof_genes = [rng.standard_normal(G) * 3.0 for _ in range(5)]
    hof_fit = [float(v) for v in np.round(rng.uniform(-1.8, 1.2, size=5), 4)]
    hof = _HoF([_Ind(list(g), f) for g, f in zip(hof_genes, hof_fit)])
    ns = make_namespace(shape, hall_of_fame=hof)
    random.seed(11)
    fits = [float(ns["evaluate"](list(g))[0]) for g in inds]
    case = dict(shape=shape, random_seed=11, individuals=[g.tolist() for g in inds],
                hof_genes=[g.tolist() for g in hof_genes], hof_fitness=hof_fit, fitness=fits, games=[])
    print(f"evaluate s3: fitness={fits}", flush=True)
    with open(os.path.join(HERE, "evaluate_s3.json"), "w") as fh:
        json.dump([case], fh)


def gen_evaluate():
    """Whole evaluate(individual) (main.py:28-66) incl. the hall-of-fame shuffles."""
    cases = []
    rng = np.random.default_rng(77)
    for shape, n_ind, n_hof, dist, seed in (([6, 2, 2], 5, 0, "init", 1),
                                            ([6, 2, 2], 6, 4, "init", 2),
                                            ([6, 2, 2], 4, 3, "n3", 3),
                                            ([6, 64, 3], 3, 3, "n1", 4)):
        G = gene_count(shape)
        inds = [gen_genes(rng, dist, G) for _ in range(n_ind)]
        hof_genes = [gen_genes(rng, dist, G) for _ in range(n_hof)]
        hof_fit = [float(np.round(rng.normal() * 0.7, 4)) for _ in range(n_hof)]
        hof = _HoF([_Ind(list(g), f) for g, f in zip(hof_genes, hof_fit)]) if n_hof else _HoF([])
        ns = make_namespace(shape, hall_of_fame=hof)
        random.seed(seed)
        games = []
        orig_pe = ns["perform_episode"]

        def pe(env, left_model, right_model, render, mult, _orig=orig_pe):
            r = _orig(env, left_model, right_model, render, mult)
            games.append(dict(reward=float(r), mult=float(mult), frames=len(env.received),
                              left=type(left_model).__name__))
            return r

        ns["perform_episode"] = pe
        fits = []
        for g in inds:
            fits.append(float(ns["evaluate"](list(g))[0]))
        cases.append(dict(shape=shape, random_seed=seed, individuals=[g.tolist() for g in inds],
                          hof_genes=[g.tolist() for g in hof_genes], hof_fitness=hof_fit,
                          fitness=fits, games=games))
        print(f"evaluate {shape} hof={n_hof}: fitness={fits}", flush=True)
    with open(os.path.join(HERE, "evaluate.json"), "w") as fh:
        json.dump(cases, fh)


def _initial_rows(seed, n, G, sigma, dtype):
    """tools/harvest_hard.py initial_rows: the harvest's host-drawn generation-0 rows."""
    return (np.random.default_rng(seed).standard_normal((n, G)) * sigma).astype(dtype)


def gen_hard_cases(harvest_path, wide_keep=1500):
    """nn_hard_cases.npz: the decisions no bound settles, harvested on the GPU
    from the bench distribution (tools/harvest_hard.py), run through the REAL
    NeuralNetwork.run (numpy_nn.py:120-137) on x = (k / 2) / 160 -- the
    inference features of the doubled centroids k (utils.py:139-153)."""
    h = dict(np.load(harvest_path))
    out = {}
    for label in ("split", "wide"):
        if f"{label}__shape" not in h:
            continue
        shape = [int(v) for v in h[f"{label}__shape"]]
        seed, P, H, G, is64 = (int(v) for v in h[f"{label}__meta"])
        sigma = float(h[f"{label}__sigma"][0])
        dt = np.float64 if is64 else np.float32
        gen, is_opp, row = h[f"{label}__gen"], h[f"{label}__is_opp"], h[f"{label}__row"]
        gidx, k, idx_dev = h[f"{label}__gidx"], h[f"{label}__k"], h[f"{label}__idx_device"]
        sel = np.arange(len(gen))
        if label == "wide" and len(sel) > wide_keep:
            sel = np.sort(np.random.default_rng(5).choice(len(sel), wide_keep, replace=False))
        pop = _initial_rows(seed, P, G, sigma, dt) if (gen[sel] == 0).any() else None
        hof = _initial_rows(seed + 1, H, G, sigma, dt) if (gen[sel] == 0).any() else None
        stored = h[f"{label}__genes"]
        acts, idxs = [], []
        nets = {}
        for i in sel:
            key = (int(gen[i]), int(is_opp[i]), int(row[i]), int(gidx[i]))
            if key not in nets:
                g = stored[gidx[i]] if gidx[i] >= 0 else (hof if is_opp[i] else pop)[row[i]]
                nets[key] = ref_nn.NeuralNetwork(nodes=list(shape), weights=[float(v) for v in g], bias=True)
            net = nets[key]
            x = [float((int(v) / 2) / 160) for v in k[i]]
            try:
                net.run(x)
            except Exception:
                pass
            a = np.array(net.list_of_transitional_arrays[-1][:-1], dtype=np.float64)
            acts.append(a)
            idxs.append(int(np.argmax(a)))
            if len(nets) > 64:
                nets.clear()
        idxs = np.array(idxs, np.int32)
        print(f"{label}: {len(sel)} cases, device == reference in {int((idxs == idx_dev[sel]).sum())}", flush=True)
        out.update({f"{label}__shape": np.array(shape, np.int32), f"{label}__meta": h[f"{label}__meta"],
                    f"{label}__sigma": h[f"{label}__sigma"], f"{label}__gen": gen[sel], f"{label}__is_opp": is_opp[sel],
                    f"{label}__row": row[sel], f"{label}__gidx": gidx[sel], f"{label}__k": k[sel],
                    f"{label}__idx_device": idx_dev[sel], f"{label}__genes": stored,
                    f"{label}__total": h[f"{label}__total"], f"{label}__idx_ref": idxs,
                    f"{label}__act_ref": np.array(acts)})
    np.savez_compressed(os.path.join(HERE, "nn_hard_cases.npz"), **out)


if __name__ == "__main__":
    if sys.argv[1:2] == ["hard_cases"]:  # python make_golden.py hard_cases <harvest.npz>
        gen_hard_cases(sys.argv[2])
        sys.exit(0)
    which = sys.argv[1:] or ["nn", "helpers", "centroids", "episodes", "evaluate"]
    if "nn" in which:
        gen_nn_forward()
    if "helpers" in which:
        gen_helpers()
    if "centroids" in which:
        gen_centroids()
    if "episodes" in which:
        gen_episodes()
    if "evaluate" in which:
        gen_evaluate()
    if "episodes_s3" in which:
        gen_episodes_s3()
    if "wide_s3" in which:
        gen_wide_s3()
    if "evaluate_s3" in which:
        gen_evaluate_s3()
