"""The pixel path on the MI355X (run with -m gpu): pg_render_frames against
the oracle's render byte for byte, pg_find_stuff against the oracle's
find_stuff restatement (pinned by the reference's own obs.npy and 300
reference find_stuff calls, tests/test_oracle_golden.py), and at full size
the rendered centroids equal the analytic ones the evaluation kernels use."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

COLOURS = np.array([[144, 72, 17], [236, 236, 236], [213, 130, 74], [92, 186, 92]], np.uint8)


def _states(gpu, n, seed):
    from pong_amd import _lib as L
    from pong_amd.device import Physics
    F = {name: i for i, name in enumerate(L.STATE_FIELD_NAMES)}
    rng = np.random.default_rng(seed)
    ph = Physics(n, device=gpu)
    ph.reset(torch.tensor(rng.integers(0, 2**62, size=n, dtype=np.int64), device=gpu),
             torch.tensor((rng.random(n) < 0.3).astype(np.int32), device=gpu))
    for _ in range(int(rng.integers(40, 400))):
        ph.step(torch.tensor(rng.integers(0, 16, size=n).astype(np.uint8), device=gpu))
    s = ph.state
    # edge cases written directly: paddles at both limits, ball at the field's corners, hidden ball
    edge = [(-8, 152, 1, 0, 20), (152, -8, 1, 156, 138), (0, 144, 0, 77, 79), (-1, 151, 1, 150, 136)]
    for i, (lpy, rpy, vis, by, bx) in enumerate(edge[: n]):
        s[F["lpy"], i], s[F["rpy"], i], s[F["ball_visible"], i] = lpy, rpy, vis
        s[F["ball_y"], i], s[F["ball_x"], i] = by, bx
    return ph


def test_render_matches_oracle(gpu, oracle):
    from pong_amd import device as D
    ph = _states(gpu, 300, 1)
    frames = D.render_frames(ph.state).cpu().numpy()
    f = ph.fields()
    for i in range(300):
        st = {k: int(f[k][i]) for k in ("ball_x", "ball_y", "ball_visible", "lpy", "rpy")}
        np.testing.assert_array_equal(frames[i], oracle.render(st), err_msg=f"frame {i}")


def test_find_stuff_matches_oracle(gpu, oracle, golden):
    from pong_amd import device as D
    rng = np.random.default_rng(2)
    ph = _states(gpu, 64, 3)
    rendered = D.render_frames(ph.state).cpu().numpy()
    obs = golden("obs.npy")
    # noise frames whose bytes are mostly the colours' own channel values, so
    # pixels match some channels of a colour and not others (get_rect_quickly's
    # per-channel rule), plus a frame with no object at all
    vals = np.concatenate([COLOURS.ravel(), rng.integers(0, 256, 8).astype(np.uint8)])
    noise = vals[rng.integers(0, vals.size, size=(48, 210, 160, 3))]
    sparse = np.broadcast_to(COLOURS[0], (16, 210, 160, 3)).copy()
    for k in range(16):
        m = rng.random((210, 160, 3)) < 0.01
        sparse[k][m] = vals[rng.integers(0, vals.size, size=int(m.sum()))]
    frames = np.concatenate([rendered, obs[None], np.zeros((1, 210, 160, 3), np.uint8), noise, sparse])
    got = D.find_stuff(torch.tensor(frames, device=gpu)).cpu().numpy()
    for i in range(frames.shape[0]):
        np.testing.assert_array_equal(got[i], oracle.find_stuff(frames[i]), err_msg=f"frame {i}")
    assert np.isnan(got[rendered.shape[0] + 1]).all()
    np.testing.assert_array_equal(got[rendered.shape[0]], np.array(golden("helpers.json")["find_stuff_obs"]))


def test_rendered_centroids_equal_analytic_at_scale(gpu):
    """65 536 physics states: find_stuff(render(state)) equals the doubled-integer
    centroids the evaluation kernels feed the networks (DESIGN.md "Physics")."""
    from pong_amd import device as D
    n = 65536
    ph = _states(gpu, n, 4)
    got = D.find_stuff(D.render_frames(ph.state)).cpu().numpy()
    f = {k: v.numpy() for k, v in ph.fields().items()}
    c2 = lambda p: np.maximum(p, 0) + np.minimum(p + 15, 159)  # noqa: E731
    np.testing.assert_array_equal(got[:, 1, 0], c2(f["lpy"]) / 2)
    np.testing.assert_array_equal(got[:, 1, 1], 17.5)
    np.testing.assert_array_equal(got[:, 2, 0], c2(f["rpy"]) / 2)
    np.testing.assert_array_equal(got[:, 2, 1], 141.5)
    vis = f["ball_visible"] == 1
    np.testing.assert_array_equal(got[vis, 0, 0], f["ball_y"][vis] + 1.5)
    np.testing.assert_array_equal(got[vis, 0, 1], f["ball_x"][vis] + 0.5)
    assert np.isnan(got[~vis, 0]).all()
