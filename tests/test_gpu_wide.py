"""k_wide (pg_wide.hip): wide two-hidden-layer networks, BASELINE config 5
([6, 512, 512, 3]), against the C oracle and the one-wave-per-game general
kernel (run with -m gpu).

Bar: bit-exact scores, frames, total_frames, f64 rewards and fitness, and
per-frame actions.  k_wide evaluates numpy_nn's own f64 operation sequence
(numpy_nn.py:126-129) with k_general's sigmoid, so the two kernels agree
bit for bit, not only on the decisions.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _gene_count(shape, bias=True):
    b = 1 if bias else 0
    return sum((shape[i] + b) * shape[i + 1] for i in range(len(shape) - 1))


def _schedule(rng, n, n_games, n_opp, nn_frac=0.6):
    kinds = rng.integers(0, 3, size=(n, n_games)).astype(np.int32)
    kinds[rng.random((n, n_games)) < nn_frac] = 3
    opp = rng.integers(0, n_opp, size=(n, n_games)).astype(np.int32)
    mult = np.ones((n, n_games))
    nn = kinds == 3
    mult[nn] = np.round(rng.normal(size=nn.sum()), 3)
    return kinds, opp, mult


def _dev(a, gpu, dt):
    return torch.tensor(np.ascontiguousarray(a), dtype=dt, device=gpu)


def _eval(ev, gpu, genomes, opponents, kinds, opp, mult, **kw):
    res, trace = ev.evaluate(_dev(genomes, gpu, ev.dtype), torch.tensor(kinds, device=gpu),
                             torch.tensor(opp, device=gpu), torch.tensor(mult, device=gpu),
                             opponents=_dev(opponents, gpu, ev.dtype), **kw)
    torch.cuda.synchronize()
    return res, trace


def _same(a, b):
    for name in ("scores", "frames", "total_frames", "rewards", "fitness", "status"):
        y = b[name] if isinstance(b, dict) else getattr(b, name).cpu().numpy()
        np.testing.assert_array_equal(getattr(a, name).cpu().numpy(), y, err_msg=name)


@pytest.mark.parametrize("shape,bias,dt", [
    ([6, 16, 8, 3], True, torch.float64),
    ([6, 40, 24, 2], True, torch.float32),
    ([6, 64, 64, 3], False, torch.float64),
    ([6, 100, 130, 4], True, torch.float32),
])
def test_wide_matches_oracle(gpu, oracle, shape, bias, dt):
    from pong_amd.device import Evaluator
    rng = np.random.default_rng(sum(shape))
    G = _gene_count(shape, bias)
    n, H = 21, 5
    genomes = (rng.standard_normal((n, G)) * 2.0)
    opponents = (rng.standard_normal((H, G)) * 2.0)
    if dt == torch.float32:
        genomes = genomes.astype(np.float32).astype(np.float64)
        opponents = opponents.astype(np.float32).astype(np.float64)
    kinds, opp, mult = _schedule(rng, n, 6, H)
    ev = Evaluator(shape, bias=bias, dtype=dt, device=gpu, kernel="wide")
    res, _ = _eval(ev, gpu, genomes, opponents, kinds, opp, mult)
    ref = oracle.eval_population(genomes, shape, kinds, opp, mult, opponents=opponents, bias=bias, n_threads=8)
    _same(res, ref)
    assert int(res.counters[0]) + int(res.counters[8]) + int(res.counters[12]) == int(ref["frames"].sum())
    assert int(res.counters[3]) == n * 6


@pytest.mark.parametrize("n_games", [1, 3, 6, 7, 8])
def test_wide_equals_general_with_traces(gpu, n_games):
    """Every column count (NG = 6 and 8 instantiations, partial columns), both
    paddles' per-frame actions, against the one-wave-per-game f64 kernel."""
    from pong_amd.device import Evaluator
    shape = [6, 96, 80, 3]
    rng = np.random.default_rng(100 + n_games)
    G = _gene_count(shape)
    n, H = 13, 4
    genomes, opponents = rng.standard_normal((n, G)) * 3.0, rng.standard_normal((H, G)) * 3.0
    kinds, opp, mult = _schedule(rng, n, n_games, H, nn_frac=0.8)
    ev = Evaluator(shape, device=gpu, n_games=n_games)
    cap = 3000
    rw, tw = _eval(ev, gpu, genomes, opponents, kinds, opp, mult, kernel="wide", trace_games=n * n_games, trace_cap=cap)
    rg, tg = _eval(ev, gpu, genomes, opponents, kinds, opp, mult, kernel="general", trace_games=n * n_games,
                   trace_cap=cap)
    _same(rw, rg)
    assert torch.equal(tw, tg)
    assert torch.equal(rw.counters[1:4], rg.counters[1:4]) and int(rw.counters[8]) == 0  # tracing: no skips


def test_wide_config5_shape_matches_oracle(gpu, oracle):
    """[6, 512, 512, 3] (config 5), f32 genome storage, self-play and scripted
    games: whole evaluations equal the oracle's."""
    from pong_amd.device import Evaluator
    shape = [6, 512, 512, 3]
    rng = np.random.default_rng(512)
    G = _gene_count(shape)
    n, H = 3, 2
    genomes = (rng.standard_normal((n, G)) * 3.0).astype(np.float32).astype(np.float64)
    opponents = (rng.standard_normal((H, G)) * 3.0).astype(np.float32).astype(np.float64)
    kinds = np.array([[0, 1, 2, 3, 3, 3], [3, 3, 3, 3, 3, 3], [3, 0, 3, 1, 3, 2]], np.int32)
    opp = rng.integers(0, H, size=(n, 6)).astype(np.int32)
    mult = np.ones((n, 6))
    ev = Evaluator(shape, dtype=torch.float32, device=gpu)  # AUTO picks the wide kernel
    res, _ = _eval(ev, gpu, genomes, opponents, kinds, opp, mult)
    ref = oracle.eval_population(genomes, shape, kinds, opp, mult, opponents=opponents, n_threads=8)
    _same(res, ref)


def test_wide_selfplay_properties(gpu):
    """A few hundred genomes of the config-5 shape: deterministic, and
    permutation-equivariant (a genome's result does not depend on which
    workgroup or slot evaluated it)."""
    from pong_amd.device import Evaluator
    shape = [6, 512, 512, 3]
    G = _gene_count(shape)
    n, H = 320, 80
    gen = torch.Generator(device=gpu).manual_seed(7)
    genomes = torch.randn((n, G), generator=gen, dtype=torch.float32, device=gpu) * 3.0
    opponents = genomes[:H].contiguous()
    ev = Evaluator(shape, dtype=torch.float32, device=gpu)
    kind, opp, mult = ev.selfplay_schedule(n, H)
    r1, _ = ev.evaluate(genomes, kind, opp, mult, opponents=opponents)
    f1 = r1.fitness.clone()
    perm = torch.randperm(n, device=gpu)
    r2, _ = ev.evaluate(genomes[perm].contiguous(), kind[perm].contiguous(), opp[perm].contiguous(),
                        mult[perm].contiguous(), opponents=opponents)
    assert torch.equal(r2.fitness, f1[perm]) and torch.equal(r2.frames, r1.frames[perm])
    assert int(r1.counters[3]) == n * 6 and int(r1.counters[0]) + int(r1.counters[8]) + int(r1.counters[12]) == int(r1.frames.sum())
    # the periodic-rally jump changes nothing: the general kernel simulates every frame
    sel = torch.arange(0, n, 13, device=gpu)
    rg, _ = ev.evaluate(genomes[sel].contiguous(), kind[sel].contiguous(), opp[sel].contiguous(),
                        mult[sel].contiguous(), opponents=opponents, kernel="general")
    assert torch.equal(rg.fitness, r1.fitness[sel]) and torch.equal(rg.frames, r1.frames[sel])
    assert torch.equal(rg.scores, r1.scores[sel]) and torch.equal(rg.total_frames, r1.total_frames[sel])


def test_wide_config5_pop4096(gpu, oracle):
    """Config 5 at pop 4 096 ([6, 512, 512, 3], f32 genome storage, self-play
    schedule of BASELINE configs[4] against 1 024 hall-of-fame rows): every
    game ends and is counted, results are permutation-equivariant, a few
    genomes' whole evaluations equal the oracle's, and every decision k_wide
    logged as a near-tie (top two activations within 1e-12) is the oracle's
    numpy-order argmax (numpy_nn.py:126-131) and k_wide's own pg_wide_decide."""
    from pong_amd.device import Evaluator
    shape = [6, 512, 512, 3]
    G = _gene_count(shape)
    n, H = 4096, 1024
    gen = torch.Generator(device=gpu).manual_seed(4096)
    genomes = torch.randn((n, G), generator=gen, dtype=torch.float32, device=gpu) * 3.0
    opponents = torch.randn((H, G), generator=gen, dtype=torch.float32, device=gpu) * 3.0
    ev = Evaluator(shape, dtype=torch.float32, device=gpu)
    kind, opp, mult = ev.selfplay_schedule(n, H)
    cap = 4096
    hard = torch.zeros((cap, 8), dtype=torch.int32, device=gpu)
    r1, _ = ev.evaluate(genomes, kind, opp, mult, opponents=opponents, hard_log=hard)
    torch.cuda.synchronize()
    c = r1.counters.cpu().numpy()
    assert int(c[3]) == n * 6 and int(c[0]) + int(c[8]) + int(c[12]) == int(r1.frames.sum())
    assert int(r1.status.sum()) == 0 and bool(torch.isfinite(r1.fitness).all())
    assert int(r1.frames.min()) >= 1
    # permutation-equivariant
    perm = torch.randperm(n, device=gpu, generator=torch.Generator(device=gpu).manual_seed(1))
    r2, _ = ev.evaluate(genomes[perm].contiguous(), kind[perm].contiguous(), opp[perm].contiguous(),
                        mult[perm].contiguous(), opponents=opponents)
    assert torch.equal(r2.fitness, r1.fitness[perm]) and torch.equal(r2.frames, r1.frames[perm])
    assert torch.equal(r2.scores, r1.scores[perm])
    # oracle re-check of four genomes: the first, the last, the longest and the fittest
    pick = sorted({0, n - 1, int(r1.frames.sum(dim=1).argmax()), int(r1.fitness.argmax())})
    sel = torch.tensor(pick, device=gpu)
    o_rows = torch.unique(opp[sel].flatten())
    remap = torch.full((H,), -1, dtype=torch.int32, device=gpu)
    remap[o_rows] = torch.arange(len(o_rows), dtype=torch.int32, device=gpu)
    ref = oracle.eval_population(genomes[sel].double().cpu().numpy(), shape, kind[sel].cpu().numpy(),
                                 remap[opp[sel].long()].cpu().numpy(), mult[sel].cpu().numpy(),
                                 opponents=opponents[o_rows].double().cpu().numpy(), n_threads=8)
    for name in ("scores", "frames", "total_frames", "rewards", "fitness"):
        np.testing.assert_array_equal(getattr(r1, name)[sel].cpu().numpy(), ref[name], err_msg=name)
    # the near-ties: the oracle's forward, and k_wide's own decision on the same input
    k = min(int(c[9]), cap)
    print(f"config 5 pop {n}: {int(c[0])} stepped + {int(c[8]) + int(c[12])} advanced frames, {int(c[9])} near-ties")
    if k:
        log = hard[:k].cpu().numpy()
        row, is_opp, idx = log[:, 0], log[:, 1] & 1, (log[:, 1] >> 8) & 255
        kk = log[:, 2:8].astype(np.int32)
        use = np.arange(k)[:512]
        for i in use:
            net = (opponents if is_opp[i] else genomes)[int(row[i])].double().cpu().numpy()
            oi, _ = oracle.nn_run(net, shape, (kk[i].astype(np.float64) / 2) / 160)
            assert oi == idx[i], (i, oi, idx[i])
        # pg_wide_decide on genome rows / opponent rows separately
        for flag, table in ((0, genomes), (1, opponents)):
            m = is_opp[use] == flag
            if not m.any():
                continue
            rows_t = torch.tensor(row[use][m], dtype=torch.int32, device=gpu)
            wi, _ = ev.wide_decide(table, torch.tensor(kk[use][m], device=gpu), genome_index=rows_t)
            np.testing.assert_array_equal(wi.cpu().numpy(), idx[use][m])
