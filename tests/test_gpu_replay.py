"""Replays and human play (run with -m gpu).

* replay.replay: the traced actions stepped through the SoA stepper and
  rasterised on the device -- every frame equal, byte for byte, to the
  oracle's own frame (or_render) of the oracle's own game (or_play_game's
  actions stepped through or_env_step); main.evaluate(render=True) writes the
  games as GIFs (render_game, main.py:115-125, headless).
* run_against_human (main.py:17-25, play_against_human.py): a HumanInput
  whose keys come from a script drives the left paddle frame by frame against
  the individual's network (perform_episode_stepwise on a DeviceEnv) -- equal
  to the reference's per-frame loop restated over the oracle's physics and
  frames (oracle/numpy_loop.perform_episode) with the same scripted keys.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_replay_reproduces_the_evaluation(gpu):
    from pong_amd import device as D
    from pong_amd import replay
    shape = [6, 16, 3]
    rng = np.random.default_rng(8)
    ev = D.Evaluator(shape, device=gpu, seed=3)
    genome = torch.tensor(rng.standard_normal(ev.genes) * 2.0, device=gpu)
    opponents = torch.tensor(rng.standard_normal((2, ev.genes)) * 2.0, device=gpu)
    kind, opp, mult = [0, 1, 2, 3, 3, 3], [0, 0, 0, 1, 0, 1], [1.0, 1.0, 1.0, 0.5, 2.0, 0.5]
    res, frames = replay.replay(ev, genome, kind, opp, mult, opponents=opponents)
    n = res.frames[0].cpu().numpy()
    assert [f.shape[0] for f in frames] == n.tolist()
    # the last frame of every game shows both paddles where find_stuff expects them
    last = torch.tensor(np.stack([f[-1] for f in frames]), device=gpu)
    c = D.find_stuff(last).cpu().numpy()
    assert not np.isnan(c[:, 1:]).any()
    assert np.all(c[:, 1, 1] == 17.5) and np.all(c[:, 2, 1] == 141.5)


def test_evaluate_render_writes_gifs(gpu, tmp_path, monkeypatch):
    import config
    import main
    monkeypatch.setattr(main, "REPLAY_DIR", str(tmp_path / "replays"), raising=False)
    monkeypatch.setattr(config, "REPLAY_DIR", str(tmp_path / "replays"))
    rng = np.random.default_rng(0)
    individual = list(rng.random(20))  # NETWORK_SHAPE [6, 2, 2]
    saved = main.hall_of_fame
    try:
        main.hall_of_fame = None
        plain = main.evaluate(individual)
        shown = main.evaluate(individual, render=True)
    finally:
        main.hall_of_fame = saved
    assert plain == shown
    files = sorted(os.listdir(tmp_path / "replays"))
    assert files == [f"game_{g}.gif" for g in range(6)]


def _oracle_frames(oracle, genes, shape, kind, opp_genes, mult, seed):
    """The oracle's game and its frames: or_play_game's traced actions stepped
    through or_env_step, each state rasterised by or_render."""
    r = oracle.play_game(genes, shape, kind, opp_genes, mult, seed, trace_cap=20000)
    tr = r["trace"]
    env = oracle.Env(seed, kind == oracle.OPP_ROM_CPU)
    frames = []
    for t in range(r["frames"]):
        prev = int(tr[t - 1]) if t >= 1 else 0  # env.step at frame t + 1 applies frame t's decision
        rc, lc = prev & 3, (prev >> 2) & 3
        env.step4(rc == 1, rc == 2, lc == 1, lc == 2)
        frames.append(oracle.render(env.snapshot()))
    return r, np.stack(frames)


@pytest.mark.parametrize("shape,sigma", [([6, 16, 3], 2.0), ([6, 64, 3], 3.0)])
def test_replay_frames_equal_oracle_frames(gpu, oracle, shape, sigma):
    from pong_amd import device as D
    from pong_amd import replay
    rng = np.random.default_rng(len(shape) + shape[1])
    ev = D.Evaluator(shape, device=gpu, seed=5)
    g_np = rng.standard_normal(ev.genes) * sigma
    o_np = rng.standard_normal((2, ev.genes)) * sigma
    kind, opp, mult = [0, 1, 2, 3, 3, 3], [0, 0, 0, 1, 0, 1], [1.0, 1.0, 1.0, 0.5, 2.0, 0.5]
    res, frames = replay.replay(ev, torch.tensor(g_np, device=gpu), kind, opp, mult,
                                opponents=torch.tensor(o_np, device=gpu))
    for g in range(6):
        r, want = _oracle_frames(oracle, g_np, shape, kind[g], o_np[opp[g]] if kind[g] == 3 else None, mult[g],
                                 oracle.game_seed(ev.seed, g))
        assert frames[g].shape == want.shape, (g, frames[g].shape, want.shape)
        bad = np.nonzero((frames[g] != want).reshape(want.shape[0], -1).any(axis=1))[0]
        assert bad.size == 0, f"game {g}: frames {bad[:5]} differ from the oracle's"
        assert float(res.rewards[0, g]) == r["reward"]
        assert (int(res.scores[0, g, 0]), int(res.scores[0, g, 1])) == (r["score1"], r["score2"])


def _scripted_keys():
    """Two key sources: a tracker with a dead zone that lets go every 97th
    call (a human-like lapse), and a fixed pattern of held keys."""
    def tracker(frame, x):
        if frame % 97 < 6:
            return 0, 0
        by, me = x[1], x[4]
        return int(by < me - 0.02), int(by > me + 0.02)
    pattern = [(1, 0)] * 20 + [(0, 0)] * 7 + [(0, 1)] * 25 + [(1, 1)] * 3
    return [("tracker", lambda: tracker), ("pattern", lambda: pattern * 400)]


@pytest.mark.parametrize("source", [0, 1])
def test_run_against_human_matches_reference_loop(gpu, source):
    """main.run_against_human with a scripted HumanInput vs the reference's
    per-frame loop (numpy_loop.perform_episode over the oracle's physics and
    frames, NumpyNet = numpy_nn.NeuralNetwork.run) with the same keys: the same
    reward, the same number of human decisions."""
    import sys
    import main
    from human_control import HumanInput
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import numpy_loop as NL
    import oracle as O
    name, keys = _scripted_keys()[source]
    rng = np.random.default_rng(40 + source)
    individual = list(rng.standard_normal(20) * 2.0)  # NETWORK_SHAPE [6, 2, 2]
    human = HumanInput(keys=keys())
    got = main.run_against_human(individual, human=human, render=False)
    ref_human = HumanInput(keys=keys())
    env = NL._Env(O.game_seed(main.PHYSICS_SEED, 0), 0)
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        want, frames, s1, s2, _tf = NL.perform_episode(env, ref_human, NL.NumpyNet([6, 2, 2], np.array(individual)), 1.0)
    assert human.frame == ref_human.frame > 0, name
    assert got == want, (name, got, want, frames, s1, s2)


def test_stepwise_equals_one_launch(gpu):
    """perform_episode frame by frame (host loop: env.step, find_stuff,
    get_actions) equals the one-launch game of the kernel for the models both
    can play: HardcodedAi, ScoreHardcodedAi and a network on the left."""
    import main
    from dumb_ais import HardcodedAi, ScoreHardcodedAi
    from numpy_nn import NeuralNetwork
    rng = np.random.default_rng(9)
    right = NeuralNetwork([6, 2, 2], bias=True, weights=list(rng.standard_normal(20) * 2.0))
    for game, left in ((0, HardcodedAi()), (2, ScoreHardcodedAi()),
                       (3, NeuralNetwork([6, 2, 2], bias=True, weights=list(rng.standard_normal(20) * 2.0)))):
        env = main.make_env(game, players=2)
        one = main.perform_episode(env, left, right, False, 0.5)
        env.reset()
        step = main.perform_episode_stepwise(env, left, right, False, 0.5)
        assert one == step, (game, one, step)
