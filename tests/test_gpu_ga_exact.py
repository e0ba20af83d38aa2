"""The device GA operators pinned by exact arithmetic (A11 / (f)1): from the
same counter-based draws (tests/_ga_draws.py restates pong_ga.hip's keys in
numpy), DEAP's own operator code -- pong_amd.deap_compat.tools.cxBlend and
mutGaussian, restated from DEAP (ga.py:89-92), driven by a stub ``random``
that hands them those draws -- gives every offspring gene of pg_ga_vary bit
for bit, and an exact rank-order computation gives every winner of
pg_ga_select_tournament_ranked / pg_ga_select_ranked (selTournament, ga.py:94)
and of the draw-by-draw pg_ga_select_tournament.  DEAP's Mersenne-Twister
stream itself is not reproduced (DEAP is absent offline); the distribution
tests are in test_gpu_ga.py."""
import numpy as np
import pytest
import torch

from _ga_draws import StubRandom, rng_key, rng_u01, splitmix64, u01

pytestmark = pytest.mark.gpu

SEED, GEN = 1234, 7
# config.py's GA parameters (ga.py:89-92, main.py:165-170)
CXPB, MUTPB, ALPHA, MU, SIGMA, INDPB = 0.9, 0.9, 0.9, 0.0, 0.9, 0.9


def _gaussians(gpu, n, G):
    """The device's Box-Muller draws of pair j, gene g: mutate zero rows with
    mu = 0, sigma = 1, indpb = 1 and no crossover, so offspring = 0 + (0 + 1 z) = z
    exactly (f64 rows); row 2j carries z_cos, row 2j + 1 z_sin."""
    from pong_amd.device import vary
    zero = torch.zeros((n, G), dtype=torch.float64, device=gpu)
    chosen = torch.arange(n, dtype=torch.int32, device=gpu)
    z, _ = vary(zero, chosen, G, 0.0, 1.0, ALPHA, 0.0, 1.0, 1.0, seed=SEED, generation=GEN)
    return z.cpu().numpy()


def _mut_draws(n):
    """Per individual: the varAnd mutation draw (random() < mutpb)."""
    return np.array([rng_u01(rng_key(SEED, GEN, 4, i), 0) for i in range(n)])


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("n", [64, 63])
def test_vary_equals_deap_operators_on_the_same_draws(gpu, monkeypatch, dtype, n):
    from pong_amd.deap_compat import tools
    from pong_amd.device import vary
    G = 643
    rng = np.random.default_rng(11)
    parents = (rng.standard_normal((97, G)) * 3.0)
    if dtype == torch.float32:
        parents = parents.astype(np.float32).astype(np.float64)
    chosen = rng.integers(0, 97, size=n).astype(np.int32)
    off, inv = vary(torch.tensor(parents, device=gpu).to(dtype), torch.tensor(chosen, device=gpu), G, CXPB, MUTPB,
                    ALPHA, MU, SIGMA, INDPB, seed=SEED, generation=GEN)
    off, inv = off.cpu().double().numpy(), inv.cpu().numpy()
    zs = _gaussians(gpu, n + (n & 1), G)
    mut = _mut_draws(n) < MUTPB
    genes = np.arange(G, dtype=np.uint64)
    n_cx = n_mut = 0
    for j in range((n + 1) // 2):
        i0, i1 = 2 * j, 2 * j + 1
        has1 = i1 < n
        ind = [list(parents[chosen[i0]]), list(parents[chosen[i1]]) if has1 else None]
        # varAnd (DEAP): clones, cxBlend of (i - 1, i) w.p. cxpb, then mutGaussian w.p. mutpb
        cx = has1 and rng_u01(rng_key(SEED, GEN, 2, j), 0) < CXPB
        if cx:
            n_cx += 1
            monkeypatch.setattr(tools, "random", StubRandom(rng_u01(rng_key(SEED, GEN, 3, j), genes)))
            tools.cxBlend(ind[0], ind[1], ALPHA)
        hb = splitmix64(rng_key(SEED, GEN, 5, j) ^ genes)
        hits = [(hb & np.uint64(0xFFFFFFFF)).astype(np.float64) * 2.0 ** -32,
                (hb >> np.uint64(32)).astype(np.float64) * 2.0 ** -32]
        for h, i in enumerate((i0, i1)):
            if i >= n:
                continue
            if mut[i]:
                n_mut += 1
                # mutGaussian draws random() for every gene and gauss() only for a hit
                gauss = zs[2 * j + h][hits[h] < INDPB]
                monkeypatch.setattr(tools, "random", StubRandom(hits[h], gauss))
                tools.mutGaussian(ind[h], MU, SIGMA, INDPB)
            want = np.array(ind[h])
            if dtype == torch.float32:
                want = want.astype(np.float32).astype(np.float64)
            assert np.array_equal(off[i, :G], want), (i, np.flatnonzero(off[i, :G] != want)[:5])
            assert inv[i] == int(cx or mut[i])
    assert n_cx > 0 and n_mut > 0


def _ranked_expected(fit, k, t, seed, gen):
    n = fit.shape[0]
    order = np.argsort(fit, kind="stable")
    srt = fit[order]
    j = np.arange(k)
    v = u01(seed, gen, 8, j, 0)
    r = np.floor(n * np.exp(np.log(v) / t)).astype(np.int64)
    r = np.clip(r, 0, n - 1)
    f = srt[r]
    lo = np.searchsorted(srt, f, "left")
    hi = np.searchsorted(srt, f, "right")
    pick = lo + np.floor(u01(seed, gen, 9, j, 0) * (hi - lo)).astype(np.int64)
    return order[np.minimum(pick, hi - 1)]


@pytest.mark.parametrize("n,t", [(4096, 1024), (1000, 7), (65536, 16384)])
def test_select_ranked_exact(gpu, n, t):
    """Rank sampling (pong_ga.h): winner rank floor(n V^(1/t)) in the stable
    ascending fitness order, the tie group's member by a second uniform --
    recomputed exactly from the same draws, with heavy ties."""
    from pong_amd import device as D
    rng = np.random.default_rng(n)
    fit = np.round(rng.standard_normal(n), 1)  # ~60 distinct values: large tie groups
    want = _ranked_expected(fit, n, t, SEED, GEN)
    ft = torch.tensor(fit, device=gpu)
    got = D.select_tournament_ranked(ft, n, t, seed=SEED, generation=GEN).cpu().numpy()
    assert np.array_equal(got, want)
    got2 = D.select_ranked(ft, n, t, SEED, GEN, D.Workspaces(gpu)).cpu().numpy()
    assert np.array_equal(got2, want)


def test_select_tournament_draw_by_draw_exact(gpu):
    """selTournament (DEAP): tournsize aspirants by selRandom, max() keeps the
    first best -- the same aspirants from the device's draws, exactly."""
    from pong_amd import device as D
    n, k, t = 500, 300, 9
    rng = np.random.default_rng(2)
    fit = np.round(rng.standard_normal(n), 1)
    got = D.select_tournament(torch.tensor(fit, device=gpu), k, t, seed=SEED, generation=GEN).cpu().numpy()
    jj, tt = np.meshgrid(np.arange(k), np.arange(t), indexing="ij")
    asp = np.floor(u01(SEED, GEN, 1, jj.ravel(), tt.ravel()) * n).astype(np.int64).reshape(k, t)
    want = asp[np.arange(k), np.argmax(fit[asp], axis=1)]  # argmax: the first maximum, as max()
    assert np.array_equal(got, want)
