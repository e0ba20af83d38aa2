"""config.py's TIMEOUT_THRESH / WIN_SCORE on the device (pg_eval_args.timeout_thresh /
win_score, ABI 11) against the oracle, on every evaluation kernel (run with -m gpu).

The threshold case of perform_episode (main.py:94-107, 128-135): a point on the
frame the no-score counter would pass TIMEOUT_THRESH resets the counter FIRST,
so the game goes on unless a score reached WIN_SCORE.  Round 5's k_service
tested the timeout before the point's reset and ended such games (round-5
review); at the reference's 2000 the case is practically unreachable in N(0, 3)
self-play (no point lands later than ~600 frames into a rally; the long ones
are periodic), at TIMEOUT_THRESH = 59 it is frequent (serve delay 30 + one
crossing: tests/test_numpy_loop.py::test_timeout_points_exist_at_thresh_59).
"""
import numpy as np
import pytest
import torch

from test_gpu_parity import _assert_same, _dev_genomes, _gene_count, _schedule

pytestmark = pytest.mark.gpu

LIMITS = [(59, 0), (119, 0), (0, 1), (0, 2), (59, 5), (2000, 3)]


def _run(ev, oracle, gpu, genomes, opponents, kinds, opp, mult, thresh, win, horizon=0):
    dt = ev.dtype
    res, _ = ev.evaluate(_dev_genomes(genomes, gpu, dt), torch.tensor(kinds, device=gpu),
                         torch.tensor(opp, device=gpu), torch.tensor(mult, device=gpu),
                         opponents=_dev_genomes(opponents, gpu, dt))
    torch.cuda.synchronize()
    ref = oracle.eval_population(genomes, ev.nodes, kinds, opp, mult, opponents=opponents, bias=ev.bias,
                                 base_seed=ev.seed, n_threads=8, horizon=horizon, timeout_thresh=thresh,
                                 win_score=win)
    return res, ref


@pytest.mark.parametrize("thresh,win", LIMITS)
@pytest.mark.parametrize("kernel,lanes", [("split", 0), ("split", 16), ("general", 0)])
def test_limits_match_oracle(gpu, oracle, kernel, lanes, thresh, win):
    from pong_amd.device import Evaluator
    shape = [6, 64, 3]
    rng = np.random.default_rng(thresh * 10 + win)
    G = _gene_count(shape)
    n, H = 256 if kernel == "split" else 64, 32
    genomes = rng.standard_normal((n, G)) * 3.0
    opponents = rng.standard_normal((H, G)) * 3.0
    kinds, opp, mult = _schedule(rng, n, 6, H)
    kinds[: n // 2] = 3  # half the population in all-network games
    ev = Evaluator(shape, device=gpu, kernel=kernel, group_lanes=lanes,
                   precision="f64" if kernel == "general" else "certified", timeout_thresh=thresh, win_score=win)
    res, ref = _run(ev, oracle, gpu, genomes, opponents, kinds, opp, mult, thresh, win)
    _assert_same(res, ref)
    if win:
        assert int(res.scores.max()) <= win


@pytest.mark.parametrize("thresh,win", [(59, 0), (119, 2)])
def test_limits_horizon_matches_oracle(gpu, oracle, thresh, win):
    """The fixed-horizon instance (auto-reset at each episode's end) under the
    limits: the round-5 code scored such a point as no episode end while its
    stale timeout test still closed the slot before T frames."""
    from pong_amd.device import Evaluator
    shape = [6, 64, 3]
    T = 1000
    rng = np.random.default_rng(thresh + 7 * win)
    G = _gene_count(shape)
    n, H = 128, 32
    genomes = rng.standard_normal((n, G)) * 3.0
    opponents = rng.standard_normal((H, G)) * 3.0
    kinds, opp, mult = _schedule(rng, n, 6, H)
    kinds[: n // 2] = 3
    ev = Evaluator(shape, device=gpu, horizon=T, timeout_thresh=thresh, win_score=win)
    res, ref = _run(ev, oracle, gpu, genomes, opponents, kinds, opp, mult, thresh, win, horizon=T)
    _assert_same(res, ref)
    assert (res.frames.cpu().numpy() == T).all()


@pytest.mark.parametrize("thresh,win", [(59, 0), (0, 1)])
def test_limits_wide_matches_oracle(gpu, oracle, thresh, win):
    from pong_amd.device import Evaluator
    shape = [6, 64, 64, 3]
    rng = np.random.default_rng(thresh + win + 1)
    G = _gene_count(shape)
    n, H = 24, 6
    genomes = rng.standard_normal((n, G)) * 2.0
    opponents = rng.standard_normal((H, G)) * 2.0
    kinds, opp, mult = _schedule(rng, n, 6, H)
    ev = Evaluator(shape, device=gpu, kernel="wide", timeout_thresh=thresh, win_score=win)
    res, ref = _run(ev, oracle, gpu, genomes, opponents, kinds, opp, mult, thresh, win)
    _assert_same(res, ref)


def test_limits_refused_out_of_range(gpu):
    from pong_amd import _lib
    from pong_amd.device import Evaluator
    shape = [6, 8, 3]
    G = _gene_count(shape)
    z = torch.zeros((2, 6), dtype=torch.int32, device=gpu)
    for thresh, win in ((31, 0), (1 << 21, 0), (0, -1)):
        ev = Evaluator(shape, device=gpu, timeout_thresh=thresh, win_score=win)
        with pytest.raises(_lib.PongGAError):
            ev.evaluate(torch.zeros((2, G), dtype=torch.float64, device=gpu), z, z,
                        torch.ones((2, 6), dtype=torch.float64, device=gpu))
