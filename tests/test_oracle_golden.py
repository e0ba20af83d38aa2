"""The CPU oracle against the reference's own outputs (CPU only).

Pins the oracle before it is trusted as the checker of the HIP path:
  * NeuralNetwork.run fixtures (numpy_nn.py:120-137), five shapes, five gene
    distributions: argmax identical, activations within BLAS-order rounding;
  * 32 whole perform_episode traces (main.py:69-112) run by the REAL
    reference code over the build's physics: every action env.step received,
    final scores, frame count and the f64 reward, bit for bit;
  * evaluate() (main.py:28-66) of 18 individuals incl. hall-of-fame games:
    the host schedule (pong_amd.schedule, same random.shuffle calls) plus the
    oracle reproduce the reference fitness bit for bit;
  * centroids of rendered frames (find_stuff, utils.py:14-19) == the analytic
    centroids the kernels use.
"""
import random

import numpy as np
import pytest

KEYS = ["6x2x2", "6x64x2", "6x64x3", "6x8x8x3", "6x4x2_nobias"]


@pytest.mark.parametrize("key", KEYS)
def test_nn_forward_matches_reference(oracle, golden, key):
    g = golden("nn_forward.npz")
    shape = [int(v) for v in g[f"{key}__shape"]]
    bias = bool(g[f"{key}__bias"])
    genes, gidx, x = g[f"{key}__genes"], g[f"{key}__gidx"], g[f"{key}__x"]
    idx_ref, act_ref = g[f"{key}__idx"], g[f"{key}__act"]
    for s in range(len(x)):
        idx, act = oracle.nn_run(genes[gidx[s]], shape, x[s], bias)
        assert idx == idx_ref[s]
        np.testing.assert_allclose(act, act_ref[s], rtol=1e-13, atol=1e-15)


@pytest.mark.parametrize("name", ["nn_forward_wide.json", "nn_forward_wide_s3.json"])
def test_nn_forward_wide_matches_reference(oracle, golden, name):
    shape = [6, 512, 512, 3]
    G = sum((shape[i] + 1) * shape[i + 1] for i in range(3))
    for c in golden(name)[:2]:
        genes = (np.random.default_rng(c["seed"]).standard_normal(G) * c["sigma"]).astype(np.float32).astype(np.float64)
        idx, act = oracle.nn_run(genes, shape, np.array(c["x"]))
        assert idx == c["idx"]
        np.testing.assert_allclose(act, c["act"], rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("name", ["episodes.json", "episodes_s3.json"])
def test_episode_traces_match_reference(oracle, golden, name):
    eps = golden(name)
    assert len(eps) == (32 if name == "episodes.json" else 24)
    for ep in eps:
        opp = None if ep["opp"] is None else np.array(ep["opp"])
        r = oracle.play_game(np.array(ep["right"]), ep["shape"], ep["kind"], opp, ep["mult"],
                             oracle.game_seed(0, ep["game_index"]), trace_cap=ep["frames"] + 1)
        assert r["frames"] == ep["frames"]
        assert (r["score1"], r["score2"]) == (ep["score1"], ep["score2"])
        assert r["reward"] == ep["reward"]
        tr = r["trace"]
        # env.step at frame t+1 receives the decision of frame t
        np.testing.assert_array_equal(tr[:-1] & 3, ep["right_actions"][1:])
        np.testing.assert_array_equal((tr[:-1] >> 2) & 3, ep["left_actions"][1:])
        assert ep["right_actions"][0] == 0 and ep["left_actions"][0] == 0  # BLANK_ACTION first


class _Fit:
    def __init__(self, v):
        self.values = (v,)
        self.valid = True


class _Member(list):
    def __init__(self, genes, fit):
        super().__init__(genes)
        self.fitness = _Fit(fit)


class _HoF:
    def __init__(self, items):
        self.items = items


@pytest.mark.parametrize("name", ["evaluate.json", "evaluate_s3.json"])
def test_evaluate_matches_reference(oracle, golden, name):
    import utils
    from pong_amd import schedule
    for case in golden(name):
        shape = case["shape"]
        members = [_Member(g, f) for g, f in zip(case["hof_genes"], case["hof_fitness"])]
        hof = _HoF(members)
        random.seed(case["random_seed"])
        n = len(case["individuals"])
        kind, opp, mult, chosen = schedule.reference_schedule(n, 6, hof, utils.pick_hall_of_famer)
        opponents = np.array([list(m) for m in chosen]) if chosen else None
        r = oracle.eval_population(np.array(case["individuals"]), shape, kind, opp, mult, opponents=opponents)
        np.testing.assert_array_equal(r["fitness"], np.array(case["fitness"]))
        # per-game rewards and multipliers in call order (recorded for evaluate.json)
        games = case["games"]
        if not games:
            continue
        np.testing.assert_array_equal(r["rewards"].ravel(), [g["reward"] for g in games])
        np.testing.assert_array_equal(mult.ravel(), [g["mult"] for g in games])
        np.testing.assert_array_equal(r["frames"].ravel(), [g["frames"] for g in games])


def test_rendered_centroids_match_analytic(golden):
    """find_stuff on frames rendered from states == the kernels' doubled centroids / 2."""
    c = golden("centroids.npy")
    lpy, rpy, vis, by, bx = (c[:, i] for i in range(5))
    c2 = lambda p: np.maximum(p, 0) + np.minimum(p + 15, 159)  # noqa: E731
    np.testing.assert_array_equal(c[:, 7], c2(lpy) / 2)
    np.testing.assert_array_equal(c[:, 8], 17.5)
    np.testing.assert_array_equal(c[:, 9], c2(rpy) / 2)
    np.testing.assert_array_equal(c[:, 10], 141.5)
    v = vis == 1
    np.testing.assert_array_equal(c[v, 5], by[v] + 1.5)
    np.testing.assert_array_equal(c[v, 6], bx[v] + 0.5)
    assert np.all(c[~v, 5] == -1)


def test_obs_npy_geometry(golden):
    """The reference's own fixture (tests.py:48-57): the object rectangles the physics uses."""
    h = golden("helpers.json")
    ball, left, right = h["find_stuff_obs"]
    assert ball == [111.5, 64.5]    # 4 x 2 ball: rows 110..113, cols 64..65
    assert left == [122.5, 17.5]    # 16 x 4 paddle at cols 16..19
    assert right == [127.5, 141.5]  # 16 x 4 paddle at cols 140..143
    assert h["find_stuff_zero"] == [None, None, None]


def test_oracle_physics_invariants(oracle):
    """Bounded paddles, ball inside the field, scores only grow, serve delay honoured."""
    rng = np.random.default_rng(0)
    for seed in range(40):
        env = oracle.Env(oracle.game_seed(seed, seed % 6), one_player=bool(seed % 3 == 1))
        prev = env.snapshot()
        hidden_run = 0
        for _ in range(3000):
            a = rng.integers(0, 16)
            env.step4(a & 1, (a >> 1) & 1, (a >> 2) & 1, (a >> 3) & 1)
            s = env.snapshot()
            assert -8 <= s["lpy"] <= 152 and -8 <= s["rpy"] <= 152
            if s["ball_visible"]:
                assert 20 <= s["ball_x"] <= 138 and 0 <= s["ball_y"] <= 156
                hidden_run = 0
            else:
                hidden_run += 1
                assert hidden_run <= 30
            assert s["score1"] >= prev["score1"] and s["score2"] >= prev["score2"]
            assert s["score1"] + s["score2"] - prev["score1"] - prev["score2"] <= 1
            prev = s
            if env.done():  # 21 points: no further serve (the emulator's episode end)
                assert max(s["score1"], s["score2"]) == 21
                break


def test_oracle_find_stuff_on_reference_fixture(oracle, golden):
    """find_stuff on the reference's own obs.npy (tests.py:48-57; copied as a
    data fixture) and on a zero frame, against the real reference's outputs."""
    h = golden("helpers.json")
    obs = golden("obs.npy")
    np.testing.assert_array_equal(oracle.find_stuff(obs), np.array(h["find_stuff_obs"]))
    assert h["find_stuff_zero"] == [None, None, None]
    assert np.isnan(oracle.find_stuff(np.zeros_like(obs))).all()


def test_oracle_render_then_find_stuff_matches_reference(oracle, golden):
    """The reference's find_stuff on 300 rendered states (tests/golden/centroids.npy)
    equals the oracle's render + find_stuff restatement."""
    c = golden("centroids.npy")
    for row in c:
        lpy, rpy, vis, by, bx = (int(v) for v in row[:5])
        st = {"lpy": lpy, "rpy": rpy, "ball_visible": vis, "ball_y": by, "ball_x": bx}
        got = oracle.find_stuff(oracle.render(st))
        want = row[5:].reshape(3, 2).copy()
        if not vis:
            want[0] = np.nan
        np.testing.assert_array_equal(got, want)
