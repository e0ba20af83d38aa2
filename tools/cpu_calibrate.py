#!/usr/bin/env python3
"""Calibrate bench.py's CPU baseline (oracle/numpy_loop.py) against the real reference.

Build container only (the reference is read-only at /root/reference; it never
travels to the GPU box).  Plays the same games twice on one core:
  * the REAL reference loop -- main.py's perform_episode / get_actions /
    calculate_timeout_and_frames AST-extracted and run with the reference's own
    utils.py (find_stuff, inference, keep_within_game_bounds_please,
    calculate_reward), numpy_nn.py (NeuralNetwork.run) and dumb_ais.py, through
    tests/golden/make_golden.py's namespace and shims;
  * the restatement oracle/numpy_loop.perform_episode,
both driven by the same emulator stand-in (numpy_loop._Env: the build's C
physics and C frame, as gym-retro's step and frame are native code), and
checks that every game's reward and frame count agree, then reports both
per-frame rates.  Output: profiles/r02/cpu_calibration.json.

usage: python tools/cpu_calibrate.py [--games 24] [--out profiles/r02/cpu_calibration.json]
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import make_golden as MG  # noqa: E402  (imports the reference modules, with its shims)
import numpy_loop as NL  # noqa: E402
import oracle as O  # noqa: E402


class _CalEnv(NL._Env):
    def close(self):
        pass


def _find_stuff_once(observation):
    """utils.find_stuff (utils.py:14-19) with the reference's own get_rect_quickly
    calls made once: numpy >= 1.24 refuses the ragged np.array([None, a, b]) of
    a hidden-ball frame, which make_golden's shim answers by recomputing all
    three rects; here the three results are kept and put in the object array
    numpy < 1.24 built, so the timing carries no shim cost."""
    chopped = observation[MG.ref_config.GAME_TOP:MG.ref_config.GAME_BOTTOM, :]
    rects = [MG.ref_utils.get_rect_quickly(chopped, c) for c in
             (MG.ref_config.BALL_COLOUR, MG.ref_config.LEFT_GUY_COLOUR, MG.ref_config.RIGHT_GUY_COLOUR)]
    try:
        return np.array(rects)
    except ValueError:
        out = np.empty(3, dtype=object)
        out[:] = rects
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=24)
    ap.add_argument("--sigma", type=float, default=3.0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r02", "cpu_calibration.json"))
    a = ap.parse_args()
    shape = [6, 64, 3]
    G = sum((shape[i] + 1) * shape[i + 1] for i in range(len(shape) - 1))
    rng = np.random.default_rng(2024)
    ns = MG.make_namespace(shape)
    ns["find_stuff"] = _find_stuff_once
    ref_pe = ns["perform_episode"]
    kinds = [(0, 3, 3, 2)[i % 4] for i in range(a.games)]  # mostly network opponents, as self-play
    cases = []
    for i in range(a.games):
        cases.append((kinds[i], i % 6, rng.standard_normal(G) * a.sigma, rng.standard_normal(G) * a.sigma,
                      float(np.round(rng.normal(), 3))))

    def run(side):
        out, frames = [], 0
        np.random.seed(5)
        t0 = time.perf_counter()
        for kind, slot, right, left, mult in cases:
            env = _CalEnv(O.game_seed(0, slot), kind == 1)
            if side == "reference":
                rm = MG.ref_utils.create_model_from_genes(list(right))
                lm = (MG.ref_utils.create_model_from_genes(list(left)) if kind == 3
                      else MG.ref_dumb.ScoreHardcodedAi() if kind == 2 else MG.ref_dumb.HardcodedAi())
                n0 = 0
                steps = [0]
                orig = env.step

                def counted(action, _o=orig, _s=steps):
                    _s[0] += 1
                    return _o(action)
                env.step = counted
                r = ref_pe(env, lm, rm, False, mult if kind == 3 else 1)
                n = steps[0] - n0
            else:
                rm = NL.NumpyNet(shape, right)
                lm = (NL.NumpyNet(shape, left) if kind == 3
                      else NL.ScoreHardcoded() if kind == 2 else NL.Hardcoded())
                r, n, _s1, _s2, _tf = NL.perform_episode(env, lm, rm, mult if kind == 3 else 1.0)
            out.append((float(r), int(n)))
            frames += n
        return out, frames, time.perf_counter() - t0

    import warnings
    warnings.simplefilter("ignore")
    # alternate the two sides and keep each one's fastest pass (host noise)
    ref_s = port_s = float("inf")
    for _ in range(a.reps):
        ref, ref_frames, t = run("reference")
        ref_s = min(ref_s, t)
        port, port_frames, t = run("restatement")
        port_s = min(port_s, t)
    agree = sum(1 for x, y in zip(ref, port) if x == y)
    res = {
        "what": "the reference's per-frame numpy loop (main.py:69-112 perform_episode with utils.find_stuff, "
                "inference, numpy_nn.NeuralNetwork.run) vs oracle/numpy_loop.py on the same games, one core, "
                "emulator stand-in = the build's C physics + C frame for both",
        "games": a.games, "passes_each": a.reps, "network_shape": shape, "genes": f"N(0,{a.sigma:g})",
        "games_agreeing": agree,
        "reference": {"frames": ref_frames, "seconds": ref_s, "env_steps_per_s": ref_frames / ref_s},
        "restatement": {"frames": port_frames, "seconds": port_s, "env_steps_per_s": port_frames / port_s},
        "restatement_over_reference": (port_frames / port_s) / (ref_frames / ref_s),
        "host": platform.processor() or platform.machine(), "numpy": np.__version__,
    }
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))
    if agree != a.games:
        sys.exit("restatement differs from the reference on %d games" % (a.games - agree))


if __name__ == "__main__":
    main()
