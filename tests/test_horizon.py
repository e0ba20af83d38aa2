"""The fixed-horizon measurement mode (pong_ga.h pg_eval_args.horizon)
in the CPU oracle (CPU only).

Every game slot runs exactly T frames; an episode that terminates before frame
T (main.py:102-107) is scored by calculate_reward and the slot auto-resets
(the serve sequence continues), the partial last episode is dropped.  Pinned
two ways:
  * at T = the frames of a REAL reference episode (tests/golden/episodes*.json,
    perform_episode run by the reference code): one completed episode with the
    reference's reward and scores; at T - 1: none;
  * a Python restatement of the auto-reset loop over the oracle's physics and
    forward (oracle.Env, oracle.nn_run) equals or_play_slot's horizon mode on
    multi-episode horizons.
"""
import numpy as np
import pytest


@pytest.mark.parametrize("name", ["episodes.json", "episodes_s3.json"])
def test_horizon_at_episode_length_is_the_reference_episode(oracle, golden, name):
    for ep in golden(name)[:16]:
        opp = None if ep["opp"] is None else np.array(ep["opp"])
        seed = oracle.game_seed(0, ep["game_index"])
        args = (np.array(ep["right"]), ep["shape"], ep["kind"], opp, ep["mult"], seed)
        r = oracle.play_game(*args, horizon=ep["frames"])
        assert r["frames"] == ep["frames"]
        assert r["total_frames"] == 1.0  # one completed episode
        assert (r["score1"], r["score2"]) == (ep["score1"], ep["score2"])
        assert r["reward"] == ep["reward"]
        r = oracle.play_game(*args, horizon=ep["frames"] - 1)
        assert r["frames"] == ep["frames"] - 1 and r["total_frames"] == 0.0 and r["reward"] == 0.0


def _restated_horizon(oracle, genes, shape, kind, opp_genes, mult, seed, T):
    """The auto-reset loop of pg_eval_args.horizon, frame by frame in Python:
    perform_episode's body (main.py:76-107) over oracle.Env, the episode
    scored by calculate_reward (utils.py:104-109) at its end, then env reset
    with the point counter kept (the serves continue)."""
    env = oracle.Env(seed, kind == 1)
    s1_tot = s2_tot = eps = 0
    reward_sum = 0.0
    zd_any = 0
    frames = 0

    def new_episode():
        return {"act_r": 0, "act_l": 0, "timeout": 0.0, "total": 0.0, "last": None, "last_ball": None}

    e = new_episode()
    while True:
        env.step4(e["act_r"] == 1, e["act_r"] == 2, e["act_l"] == 1, e["act_l"] == 2)
        frames += 1
        st = env.state
        vis = st.ball_visible
        by2, bx2 = 2 * st.ball_y + 3, 2 * st.ball_x + 1
        lc2 = max(st.lpy, 0) + min(st.lpy + 15, 159)
        rc2 = max(st.rpy, 0) + min(st.rpy + 15, 159)
        left = right = 0
        if vis:
            lby2, lbx2 = e["last_ball"] if e["last_ball"] is not None else (by2, bx2)
            xr = np.array([0.5 * bx2, 0.5 * by2, 0.5 * lbx2, 0.5 * lby2, 0.5 * rc2, 0.5 * lc2]) / 160.0
            xl = np.array([160.0 - 0.5 * bx2, 0.5 * by2, 160.0 - 0.5 * lbx2, 0.5 * lby2, 0.5 * lc2,
                           0.5 * rc2]) / 160.0
            code = {0: 1, 1: 2}
            if kind == 3:
                left = code.get(oracle.nn_run(opp_genes, shape, xl)[0], 0)
            elif kind == 2 and st.score1 > st.score2:
                left = 0
            else:
                left = 1 if xl[1] < xl[4] else (2 if xl[1] > xl[4] else 0)
            right = code.get(oracle.nn_run(genes, shape, xr)[0], 0)
        e["last_ball"] = (by2, bx2) if vis else None
        clamp = lambda c2, a: 2 if c2 < 32 else (1 if c2 > 288 else a)  # noqa: E731
        e["act_l"], e["act_r"] = clamp(lc2, left), clamp(rc2, right)
        sc = (st.score1, st.score2)
        if e["last"] is not None:
            if sc == e["last"]:
                e["timeout"] += 1.0
            else:
                e["total"] += e["timeout"]
                e["timeout"] = 0.0
        e["last"] = sc
        ep_end = max(sc) >= 3 or env.done() or e["timeout"] > 2000
        if ep_end:
            if sc[0] != sc[1]:
                if e["total"] == 0.0:
                    zd_any = 1
                    reward_sum += float("nan")
                else:
                    reward_sum += ((sc[1] - sc[0]) + sc[1] * mult) / (e["total"] / 100.0)
            eps += 1
            s1_tot += sc[0]
            s2_tot += sc[1]
            if frames >= T:
                break
            point = env.state.point
            env.reset()
            env.state.point = point
            e = new_episode()
            continue
        if frames >= T:
            s1_tot += sc[0]
            s2_tot += sc[1]
            break
    return {"frames": frames, "score1": s1_tot, "score2": s2_tot, "total_frames": float(eps),
            "reward": reward_sum, "zero_division": zd_any}


@pytest.mark.parametrize("kind", [0, 1, 2, 3])
def test_horizon_auto_reset_matches_restatement(oracle, kind):
    shape = [6, 2, 2]
    G = (6 + 1) * 2 + (2 + 1) * 2
    rng = np.random.default_rng(40 + kind)
    for trial in range(3):
        genes, opp = rng.standard_normal(G) * 3.0, rng.standard_normal(G) * 3.0
        mult = float(np.round(rng.normal(), 3)) if kind == 3 else 1.0
        seed = oracle.game_seed(1234, trial)
        T = int(rng.integers(600, 1400))
        got = oracle.play_game(genes, shape, kind, opp if kind == 3 else None, mult, seed, horizon=T)
        want = _restated_horizon(oracle, genes, shape, kind, opp, mult, seed, T)
        for k in ("frames", "score1", "score2", "total_frames", "zero_division"):
            assert got[k] == want[k], (k, got[k], want[k])
        np.testing.assert_array_equal(got["reward"], want["reward"])
        assert got["frames"] == T


def test_horizon_population_counts(oracle):
    """or_eval_population_h: frames = T everywhere, fitness = sum(rewards) / games."""
    shape = [6, 4, 3]
    G = 7 * 4 + 5 * 3
    rng = np.random.default_rng(9)
    n, H, T = 24, 5, 700
    genomes, opponents = rng.standard_normal((n, G)) * 3.0, rng.standard_normal((H, G)) * 3.0
    kinds = np.tile(np.array([0, 1, 2, 3, 3, 3], np.int32), (n, 1))
    opp = rng.integers(0, H, size=(n, 6)).astype(np.int32)
    mult = np.ones((n, 6))
    r = oracle.eval_population(genomes, shape, kinds, opp, mult, opponents=opponents, horizon=T)
    assert (r["frames"] == T).all()
    assert (r["total_frames"] >= 0).all() and r["total_frames"].sum() > 0
    np.testing.assert_array_equal(r["fitness"], np.array([sum(row) / 6.0 for row in r["rewards"].tolist()]))
