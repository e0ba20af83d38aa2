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


def _timeout_points(trace, thresh):
    """Frames of points whose no-score counter (main.py:128-135) would have
    passed ``thresh`` on that very frame: the point resets it first
    (main.py:94-107), so the game goes on unless a score reached WIN_SCORE."""
    vis = (np.asarray(trace) >> 4) & 1
    last, out = 1, []
    for f in range(2, len(vis) + 1):
        if vis[f - 2] == 1 and vis[f - 1] == 0:  # the ball vanished on frame f: a point
            if f - last == thresh + 1:
                out.append(f)
            last = f
    return out


@pytest.mark.parametrize("thresh,win", [(59, 0), (119, 0), (0, 1), (0, 2), (59, 5)])
def test_episode_limits_match_oracle(thresh, win):
    """config.py's TIMEOUT_THRESH / WIN_SCORE (pg_eval_args.timeout_thresh /
    win_score): the numpy restatement of perform_episode (main.py:69-112) and
    the C oracle agree at other values than the reference's 2000 / 3 -- in
    particular on points that land on the frame the no-score counter would
    pass the threshold (counter reset first, main.py:94-107)."""
    rng = np.random.default_rng(31 + thresh + win)
    shape = [6, 8, 3]
    G = 7 * 8 + 9 * 3
    genomes = rng.standard_normal((2, G)) * 3
    opponents = rng.standard_normal((2, G)) * 3
    kinds = np.tile(np.array([0, 1, 2, 3, 3, 3], np.int32), (2, 1))
    opp = rng.integers(0, 2, (2, 6)).astype(np.int32)
    mult = np.where(kinds == 3, 0.7, 1.0)
    ref = O.eval_population(genomes, shape, kinds, opp, mult, opponents=opponents, timeout_thresh=thresh,
                            win_score=win)
    for i in range(2):
        fit, rew, frames = NL.evaluate(shape, genomes[i], kinds[i], opp[i], mult[i], opponents,
                                       timeout_thresh=thresh or None, win_score=win or None)
        np.testing.assert_array_equal(np.array(rew, dtype=np.float64), ref["rewards"][i])
        assert fit == ref["fitness"][i]
        assert frames == int(ref["frames"][i].sum())
    if win:
        assert ref["scores"].max() <= max(win, 1)
    # the limits are restored after the call
    d = O.eval_population(genomes[:1], shape, kinds[:1], opp[:1], mult[:1], opponents=opponents)
    d0 = O.eval_population(genomes[:1], shape, kinds[:1], opp[:1], mult[:1], opponents=opponents,
                           timeout_thresh=2000, win_score=3)
    np.testing.assert_array_equal(d["frames"], d0["frames"])


def test_timeout_points_exist_at_thresh_59():
    """The GPU limit tests (test_gpu_limits.py) run at TIMEOUT_THRESH = 59
    because N(0, 3) self-play puts points on the 60th frame of a rally often
    (serve delay 30 + a crossing): the threshold case is exercised, and the
    oracle plays on past it."""
    rng = np.random.default_rng(3)
    G = 7 * 64 + 65 * 3
    n_ev = 0
    for i in range(12):
        r, l_ = rng.standard_normal(G) * 3, rng.standard_normal(G) * 3
        for g in range(6):
            res = O.play_game(r, [6, 64, 3], O.OPP_NN, l_, 1.0, O.game_seed(0, g), trace_cap=20000,
                              timeout_thresh=59)
            ev = _timeout_points(res["trace"], 59)
            n_ev += sum(1 for f in ev if f < res["frames"])
    assert n_ev > 0
