"""The decisions no bound settles, replayed on the MI355X (run with -m gpu).

tests/golden/nn_hard_cases.npz holds the forwards the hot kernel's certified
cascade handed to its numpy-order f64 forward on the bench distribution, and
k_wide's near-tie decisions, with the REAL reference's NeuralNetwork.run
answers (numpy_nn.py:120-137).  pg_decide runs k_service's very cascade on
them, pg_wide_decide runs k_wide itself; pg_forward's f64 path is the
k_general arithmetic."""
import numpy as np
import pytest
import torch

from _hard_cases import load

pytestmark = pytest.mark.gpu


def test_split_hard_cases_decide_as_numpy(gpu):
    from pong_amd.device import Evaluator
    c = load("split")
    ev = Evaluator(c["shape"], device=gpu)
    g = torch.tensor(c["genes"], device=gpu)
    idx, stage = ev.decide(g, torch.tensor(c["k"], device=gpu))
    np.testing.assert_array_equal(idx.cpu().numpy(), c["idx_ref"])
    st = np.bincount(stage.cpu().numpy(), minlength=5)
    print(f"{len(c['idx_ref'])} hard cases, stages {st.tolist()}")
    # they are the numpy-order forward's cases (the frame's own bound, stage 4,
    # may settle a plateau tie among them first)
    assert st[3] + st[4] > 0.9 * st.sum()
    i64, act = ev.forward(g, torch.tensor(c["x"], device=gpu), precision="f64")
    np.testing.assert_array_equal(i64.cpu().numpy(), c["idx_ref"])
    np.testing.assert_allclose(act.cpu().numpy(), c["act_ref"], rtol=0, atol=1e-12)


def test_wide_near_ties_decide_as_numpy(gpu):
    from pong_amd.device import Evaluator
    c = load("wide")
    ev = Evaluator(c["shape"], device=gpu, precision="f64")
    n = len(c["idx_ref"])
    for s in range(0, n, 256):
        g = torch.tensor(c["genes"][s:s + 256], device=gpu)
        idx, act = ev.forward(g, torch.tensor(c["x"][s:s + 256], device=gpu))
        np.testing.assert_array_equal(idx.cpu().numpy(), c["idx_ref"][s:s + 256])
        np.testing.assert_allclose(act.cpu().numpy(), c["act_ref"][s:s + 256], rtol=0, atol=1e-12)


@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
def test_wide_near_ties_through_k_wide(gpu, dt):
    """The 1 500 near-ties k_wide logged on the config-5 bench distribution,
    replayed through k_wide ITSELF (pg_wide_decide: one frame of the
    evaluation kernel per case, its layer path and argmax): the reference's
    NeuralNetwork.run argmax every time.  The harvest stored f32 genomes, so
    both storage widths hold the same weights."""
    from pong_amd.device import Evaluator
    c = load("wide")
    ev = Evaluator(c["shape"], dtype=dt, device=gpu)
    n = len(c["idx_ref"])
    for s in range(0, n, 256):
        g = torch.tensor(c["genes"][s:s + 256], dtype=dt, device=gpu)
        idx, act = ev.wide_decide(g, torch.tensor(c["k"][s:s + 256], device=gpu))
        np.testing.assert_array_equal(idx.cpu().numpy(), c["idx_ref"][s:s + 256])
        np.testing.assert_allclose(act.cpu().numpy(), c["act_ref"][s:s + 256], rtol=0, atol=1e-12)
        np.testing.assert_array_equal(idx.cpu().numpy(), c["idx_device"][s:s + 256])
