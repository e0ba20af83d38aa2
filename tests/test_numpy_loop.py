"""The CPU baseline's numpy loop (oracle/numpy_loop.py) against the reference.

numpy_loop restates the reference's per-frame numpy path (main.py:69-112,
utils.py:14-19/139-153, numpy_nn.py:120-137); bench.py times it as the
cpu_baseline.  Pinned here to the real reference's episode traces
(tests/golden/episodes.json, written by make_golden.py from the reference's own
perform_episode) and to the C oracle's whole-population evaluate.
"""
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import numpy_loop as NL  # noqa: E402
import oracle as O  # noqa: E402

pytestmark = pytest.mark.filterwarnings("ignore::RuntimeWarning")


def _episodes():
    with open(os.path.join(HERE, "golden", "episodes.json")) as fh:
        return json.load(fh)


def _episodes_s3():
    with open(os.path.join(HERE, "golden", "episodes_s3.json")) as fh:
        return json.load(fh)


@pytest.mark.parametrize("case", [("episodes.json", i) for i in range(0, 32, 3)] +
                         [("episodes_s3.json", i) for i in (0, 3, 5)])
def test_perform_episode_matches_reference_trace(case):
    name, i = case
    ep = (_episodes() if name == "episodes.json" else _episodes_s3())[i]
    shape, kind = ep["shape"], ep["kind"]
    right = NL.NumpyNet(shape, np.array(ep["right"]))
    left = (NL.NumpyNet(shape, np.array(ep["opp"])) if kind == O.OPP_NN
            else NL.ScoreHardcoded() if kind == O.OPP_SCORE else NL.Hardcoded())
    env = NL._Env(O.game_seed(0, ep["game_index"]), kind == O.OPP_ROM_CPU)
    reward, frames, s1, s2, _tf = NL.perform_episode(env, left, right, ep["mult"] if kind == O.OPP_NN else 1.0)
    assert frames == ep["frames"]
    assert (s1, s2) == (ep["score1"], ep["score2"])
    assert float(reward) == ep["reward"]


def test_evaluate_matches_oracle_population():
    rng = np.random.default_rng(11)
    shape = [6, 8, 3]
    G = 7 * 8 + 9 * 3
    genomes = rng.standard_normal((3, G)) * 3
    opponents = rng.standard_normal((2, G)) * 3
    kinds = np.tile(np.array([0, 1, 2, 3, 3, 3], np.int32), (3, 1))
    opp = rng.integers(0, 2, (3, 6)).astype(np.int32)
    mult = np.where(kinds == 3, 0.7, 1.0)
    ref = O.eval_population(genomes, shape, kinds, opp, mult, opponents=opponents)
    for i in range(3):
        fit, _rew, frames = NL.evaluate(shape, genomes[i], kinds[i], opp[i], mult[i], opponents)
        assert fit == ref["fitness"][i]
        assert frames == int(ref["frames"][i].sum())


def test_timed_rate_pool():
    rng = np.random.default_rng(12)
    shape = [6, 8, 3]
    G = 7 * 8 + 9 * 3
    genomes = rng.standard_normal((4, G))
    kinds = np.full((4, 6), 3, np.int32)
    opp = np.zeros((4, 6), np.int32)
    mult = np.ones((4, 6))
    rate, steps, games, dt = NL.timed_rate(shape, genomes, kinds, opp, mult, genomes[:1], 1.0, workers=2)
    assert steps > 0 and games > 0 and rate > 0


def test_timed_rate_solo_leg_same_sample():
    """The one-core leg replays worker 0's games alone: same games from the start."""
    import numpy as np
    import numpy_loop as NL
    shape = [6, 2, 2]
    rng = np.random.default_rng(5)
    genomes = rng.standard_normal((4, 20))
    kinds = np.zeros((4, 6), np.int32)
    opp = np.zeros((4, 6), np.int32)
    mult = np.ones((4, 6))
    out = NL.timed_rate(shape, genomes, kinds, opp, mult, genomes[:1], 0.5, workers=2, solo_seconds=0.5)
    assert len(out) == 5
    rate_s, steps_s, games_s, dt_s, w0 = out[4]
    assert rate_s > 0 and steps_s > 0 and games_s > 0 and w0 > 0
