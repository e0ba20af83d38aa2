"""The frame bound of k_service's residual (pg_cascade.hpp frame_bound) on CPU.

frame_bound replaces load_net_pk's worst-case magnitudes (|x_i| <= 1, sigmoid
slope <= 1/4, s_j <= 1) by the frame's own, so certificate failures that the
network's static bound leaves to the f64 stage can still be decided in f32.
Its soundness is what the kernel's decisions rest on; this restates both
bounds in numpy over an f32 emulation of partial_pk (pre-scaled weights, the
fma chain rounded once per step, exp2 / +1 / reciprocal each rounded to f32)
and checks, on random [6, 64, 3] networks of the bench's N(0, sigma) genes and
random features, that
  * the f32 outputs stay within the frame bound of the f64 outputs
    (numpy_nn.py:120-137's z), with the bound's x2 margin untouched, and
  * the frame bound never exceeds the static one (the kernel takes the min),
    and is several times tighter for the bench's sigma = 3 networks.
numpy's f32 division is correctly rounded and its exp2 within an ulp, as
v_exp_f32 / v_rcp_f32 are within ~1 ulp; the bound budgets 5u relative for
the sigmoid's three roundings, so the emulation sits inside the hardware's
error model.
"""
import numpy as np
import pytest

f32 = np.float32
U = 2.0 ** -24
L2E = 1.4426950408889634
OR = 8 + 2 + 3  # out_roundings<4, 16>: 8 chained pk_fma, log2(4) tree levels, + 3


def _nets(rng, n, H, sigma):
    return (rng.standard_normal((n, H, 7)) * sigma, rng.standard_normal((n, 3, H)) * sigma,
            rng.standard_normal((n, 3)) * sigma)


def _check(sigma, n_nets=200, frames=64, H=64, seed=1):
    rng = np.random.default_rng(seed)
    W1s, W2s, cs = _nets(rng, n_nets, H, sigma)
    worst, ratios = 0.0, []
    for W1, W2, c in zip(W1s, W2s, cs):
        k = rng.integers(0, 321, size=(frames, 6)).astype(np.float64)
        x = np.concatenate([k / 320.0, np.ones((frames, 1))], 1)
        z = 1 / (1 + np.exp(-(x @ W1.T))) @ W2.T + c  # f64, numpy_nn.py's forward
        # partial_pk in f32: W1 pre-scaled by -log2 e / 320 (features) and -log2 e (bias)
        w1s = np.concatenate([(W1[:, :6].astype(f32) * f32(-L2E / 320)).astype(f32),
                              (W1[:, 6:].astype(f32) * f32(-L2E)).astype(f32)], 1)
        a = np.broadcast_to(w1s[:, 6], (frames, H)).astype(f32)
        for i in range(6):  # fma: exact product and sum in f64, one rounding to f32
            a = (w1s[:, i].astype(np.float64) * k[:, i:i + 1] + a.astype(np.float64)).astype(f32)
        s = (f32(1) / (np.exp2(a).astype(f32) + f32(1)).astype(f32)).astype(f32)
        zc = s.astype(np.float64) @ W2.astype(f32).astype(np.float64).T + c.astype(f32)
        # load_net_pk's static bound
        R = np.abs(W1.astype(f32)).sum(1)
        e_static = 2 * U * max((np.abs(W2[o]) * (3 * R + 5 + OR)).sum() + OR * abs(c[o]) for o in range(3))
        # frame_bound, term by term
        r = np.abs(w1s[:, 6]) + k @ np.abs(w1s[:, :6]).T
        da = (r + np.abs(w1s).sum(1) * 320 * 2.0 ** -20) * 11 * U
        slope = np.minimum(0.25, np.exp2(2 * da - np.abs(a)))
        ds = slope * da * np.log(2) + s * (5 + OR) * U + 2.0 ** -100
        e_frame = 2 * np.max(ds @ np.abs(W2).T + OR * U * np.abs(c), 1)
        err = np.abs(zc - z).max(1)
        worst = max(worst, float((err / e_frame).max()))
        ratios.append(e_frame / e_static)
    return worst, np.concatenate(ratios)


@pytest.mark.parametrize("sigma", [3.0, 1.0, 0.3])
def test_frame_bound_sound_and_tighter(sigma):
    worst, ratio = _check(sigma)
    assert worst < 0.5, worst  # well inside the bound (the x2 margin is not needed here)
    assert ratio.max() <= 1.0
    if sigma == 3.0:
        assert np.median(ratio) < 0.35  # the bench's networks: ~4x tighter (0.26 measured)
