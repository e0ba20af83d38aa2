"""Device GA operators (pg_ga_select_tournament[_ranked], pg_ga_vary) against
the distributions of DEAP's tools.selTournament, tools.cxBlend,
tools.mutGaussian and algorithms.varAnd (ga.py:89-94).  DEAP's Mersenne
Twister stream is not reproduced on device, so these are
distribution and invariant checks; the host restatement's exact call order is
tested in test_deap_compat.py."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _fit(gpu, n, seed=0):
    rng = np.random.default_rng(seed)
    return torch.tensor(rng.standard_normal(n), dtype=torch.float64, device=gpu)


def _winner_rank_cdf(n, t):
    r = np.arange(n)
    return ((r + 1) / n) ** t  # P(winner rank <= r) for distinct fitness values


@pytest.mark.parametrize("n,t", [(64, 1), (64, 3), (1000, 7), (4096, 1024)])
def test_select_tournament_distributions(gpu, n, t):
    from pong_amd.device import select_tournament, select_tournament_ranked
    fit = _fit(gpu, n)
    k = 200_000
    ranks = torch.argsort(torch.argsort(fit)).cpu().numpy()  # ascending rank of each row
    expect = _winner_rank_cdf(n, t)
    for fn in (select_tournament, select_tournament_ranked):
        if fn is select_tournament and t > 64:
            continue  # draw-by-draw selection: O(k t)
        chosen = fn(fit, k, t, seed=3, generation=1).cpu().numpy()
        assert chosen.min() >= 0 and chosen.max() < n
        emp = np.cumsum(np.bincount(ranks[chosen], minlength=n)) / k
        assert np.abs(emp - expect).max() < 0.01, fn.__name__


def test_select_ranked_ties_uniform(gpu):
    from pong_amd.device import select_tournament_ranked
    fit = torch.zeros(128, dtype=torch.float64, device=gpu)  # one tie group
    chosen = select_tournament_ranked(fit, 128_000, 8, seed=1, generation=0).cpu().numpy()
    counts = np.bincount(chosen, minlength=128)
    assert counts.min() > 800 and counts.max() < 1200  # uniform over the tie group (1000 each)


def test_select_deterministic_per_generation(gpu):
    from pong_amd.device import select_tournament_ranked
    fit = _fit(gpu, 512)
    a = select_tournament_ranked(fit, 512, 16, seed=9, generation=4)
    b = select_tournament_ranked(fit, 512, 16, seed=9, generation=4)
    c = select_tournament_ranked(fit, 512, 16, seed=9, generation=5)
    assert torch.equal(a, b) and not torch.equal(a, c)


def _parents(gpu, n, g, dtype=torch.float64):
    return torch.randn((n, g), generator=torch.Generator(device=gpu).manual_seed(0), dtype=torch.float64,
                       device=gpu).to(dtype)


def test_vary_identity_without_operators(gpu):
    from pong_amd.device import vary
    par = _parents(gpu, 300, 70)
    chosen = torch.randint(0, 300, (301,), dtype=torch.int32, device=gpu)
    off, inv = vary(par, chosen, 70, 0.0, 0.0, 0.9, 0.0, 0.9, 0.9, seed=1, generation=0)
    assert torch.equal(off, par[chosen.long()]) and int(inv.sum()) == 0


def test_vary_blend_is_affine_and_preserves_pair_sums(gpu):
    """cxBlend: x1' + x2' = x1 + x2 (up to rounding), gamma in [-alpha, 1 + alpha]."""
    from pong_amd.device import vary
    par = _parents(gpu, 64, 500)
    chosen = torch.arange(64, dtype=torch.int32, device=gpu)
    alpha = 0.5
    off, inv = vary(par, chosen, 500, 1.0, 0.0, alpha, 0.0, 1.0, 1.0, seed=2, generation=0)
    x1, x2 = par[0::2], par[1::2]
    y1, y2 = off[0::2], off[1::2]
    torch.testing.assert_close(y1 + y2, x1 + x2, rtol=0, atol=1e-12)
    gamma = ((y2 - x1) / (x2 - x1)).cpu().numpy()  # y2 = gamma x1 + (1-gamma) x2  ->  1 - gamma
    g = 1.0 - gamma
    ok = np.abs((x2 - x1).cpu().numpy()) > 1e-3
    assert g[ok].min() >= -alpha - 1e-6 and g[ok].max() <= 1 + alpha + 1e-6
    assert abs(g[ok].mean() - 0.5) < 0.02  # U[-alpha, 1+alpha] has mean 1/2
    assert int(inv.sum()) == 64


@pytest.mark.parametrize("indpb", [1.0, 0.3])
def test_vary_gaussian_mutation_moments(gpu, indpb):
    from pong_amd.device import vary
    n, g = 256, 2000
    par = _parents(gpu, n, g)
    chosen = torch.arange(n, dtype=torch.int32, device=gpu)
    mu, sigma = 0.25, 0.9
    off, inv = vary(par, chosen, g, 0.0, 1.0, 0.9, mu, sigma, indpb, seed=5, generation=2)
    d = (off - par).cpu().numpy().ravel()
    moved = d != 0
    assert abs(moved.mean() - indpb) < 0.01
    dm = d[moved]
    assert abs(dm.mean() - mu) < 0.01 and abs(dm.std() - sigma) < 0.01
    # normality: fraction within one sigma of the mean
    assert abs((np.abs(dm - mu) < sigma).mean() - 0.6827) < 0.01
    assert int(inv.sum()) == n


def test_vary_mutpb_fraction_and_f32(gpu):
    from pong_amd.device import vary
    n, g = 4000, 16
    par = _parents(gpu, n, g, torch.float32)
    chosen = torch.arange(n, dtype=torch.int32, device=gpu)
    off, inv = vary(par, chosen, g, 0.0, 0.4, 0.9, 0.0, 1.0, 1.0, seed=6, generation=0)
    changed = (off != par).any(dim=1).cpu().numpy()
    assert abs(changed.mean() - 0.4) < 0.03
    np.testing.assert_array_equal(changed, inv.cpu().numpy().astype(bool))


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_gather_rows_applies_hof_sources(gpu, dtype):
    """pg_gather_rows: dst[j] = old[src[j]] below n_old, else rows[index[src[j] - n_old]]."""
    from pong_amd import device as D
    rng = np.random.default_rng(5)
    G, n_old, n_rows = 643, 37, 90
    store = torch.randn((n_old + 200, G + 5), dtype=torch.float64, device=gpu).to(dtype)  # wider stride
    rows = torch.randn((n_rows, G), dtype=torch.float64, device=gpu).to(dtype)
    cand = torch.tensor(rng.permutation(n_rows)[:50], dtype=torch.int64, device=gpu)
    src = rng.integers(0, n_old + 50, size=61).astype(np.int32)
    dst = torch.zeros((64, G), dtype=dtype, device=gpu)
    D.gather_rows(dst, store, rows, torch.tensor(src, device=gpu), n_old, index=cand, genes=G)
    want = torch.stack([store[s, :G] if s < n_old else rows[cand[s - n_old]] for s in src.tolist()])
    assert torch.equal(dst[:61], want) and bool((dst[61:] == 0).all())
    # without an index the population entry is the row itself
    D.gather_rows(dst, store, rows, torch.tensor(src, device=gpu), n_old, genes=G)
    want = torch.stack([store[s, :G] if s < n_old else rows[s - n_old] for s in src.tolist()])
    assert torch.equal(dst[:61], want)
