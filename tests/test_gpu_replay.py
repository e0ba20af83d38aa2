"""Replays (run with -m gpu): the traced actions stepped through the SoA
stepper end every game at the evaluation's score and frame count, and
main.evaluate(render=True) writes the games as GIFs (render_game,
main.py:115-125, headless)."""
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
