"""HIP path vs the CPU oracle and the reference's golden vectors (run with -m gpu).

Bar: bit-exact for actions, scores, frames and f64 rewards/fitness; final
activations within 1e-5 (certified f32 path) / 1e-12 (f64 path) of numpy_nn.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES_RES = [[6, 2, 2], [6, 64, 3], [6, 64, 2], [6, 16, 3], [6, 100, 3]]


def _dev_genomes(a, dev, dtype=torch.float64):
    return torch.tensor(np.ascontiguousarray(a), dtype=dtype, device=dev)


def _gene_count(shape, bias=True):
    b = 1 if bias else 0
    return sum((shape[i] + b) * shape[i + 1] for i in range(len(shape) - 1))


# ------------------------------------------------------------------ forward
@pytest.mark.parametrize("key", ["6x2x2", "6x64x2", "6x64x3", "6x8x8x3", "6x4x2_nobias"])
@pytest.mark.parametrize("precision", ["certified", "f64"])
def test_forward_matches_reference_golden(gpu, golden, key, precision):
    from pong_amd.device import Evaluator
    g = golden("nn_forward.npz")
    shape = [int(v) for v in g[f"{key}__shape"]]
    bias = bool(g[f"{key}__bias"])
    genes, gidx, x = g[f"{key}__genes"], g[f"{key}__gidx"], g[f"{key}__x"]
    ev = Evaluator(shape, bias=bias, device=gpu, precision=precision)
    idx, act = ev.forward(_dev_genomes(genes, gpu), torch.tensor(x, dtype=torch.float64, device=gpu),
                          genome_index=torch.tensor(gidx, dtype=torch.int32, device=gpu))
    np.testing.assert_array_equal(idx.cpu().numpy(), g[f"{key}__idx"])
    tol = 1e-5 if (precision == "certified" and len(shape) == 3) else 1e-12
    np.testing.assert_allclose(act.cpu().numpy(), g[f"{key}__act"], rtol=0, atol=tol)


@pytest.mark.parametrize("name", ["nn_forward_wide.json", "nn_forward_wide_s3.json"])
def test_forward_wide_golden(gpu, golden, name):
    """[6,512,512,3] (config 5 shape) through the general f64 path; σ 0.05 / 1
    and the wide bench's σ 3 (_s3)."""
    from pong_amd.device import Evaluator
    import hashlib
    cases = golden(name)
    shape = [6, 512, 512, 3]
    ev = Evaluator(shape, device=gpu, precision="f64")
    for c in cases:
        genes = np.random.default_rng(c["seed"]).standard_normal(_gene_count(shape)) * c["sigma"]
        genes = genes.astype(np.float32).astype(np.float64)
        assert hashlib.sha256(genes.tobytes()).hexdigest() == c["genes_sha256"]
        idx, act = ev.forward(_dev_genomes(genes[None], gpu), torch.tensor([c["x"]], dtype=torch.float64, device=gpu))
        assert int(idx[0]) == c["idx"]
        np.testing.assert_allclose(act[0].cpu().numpy(), c["act"], rtol=0, atol=1e-12)


@pytest.mark.parametrize("shape", [[6, 2, 2], [6, 64, 3], [6, 16, 2], [6, 200, 4]])
def test_forward_certified_equals_f64(gpu, oracle, shape):
    """The certified f32 argmax equals the f64 argmax on every decision (1.5M+ passes)."""
    from pong_amd.device import Evaluator
    rng = np.random.default_rng(len(shape) * 100 + shape[1])
    G = _gene_count(shape)
    ev = Evaluator(shape, device=gpu)
    n_gen, per = 2048, 192
    tot_slow = 0
    for dist in ("init", 1.0, 3.0, 9.0, 30.0):
        if dist == "init":
            genes = rng.random((n_gen, G))
        else:
            genes = rng.standard_normal((n_gen, G)) * dist
        dg = _dev_genomes(genes, gpu)
        gi = torch.tensor(np.repeat(np.arange(n_gen), per), dtype=torch.int32, device=gpu)
        k = rng.integers(0, 321, size=(n_gen * per, 6))
        x = torch.tensor(k / 320.0, dtype=torch.float64, device=gpu)
        i_cert, _ = ev.forward(dg, x, genome_index=gi, precision="certified", want_act=False)
        tot_slow += int(ev.last_forward_counters[2])
        i_f64, _ = ev.forward(dg, x, genome_index=gi, precision="f64", want_act=False)
        np.testing.assert_array_equal(i_cert.cpu().numpy(), i_f64.cpu().numpy())
        # and the oracle on a sample
        sel = rng.integers(0, n_gen * per, size=64)
        kk = k[sel]
        for s, row in zip(sel, kk):
            ref_idx, _ = oracle.nn_run(genes[s // per], shape, row / 320.0)
            assert int(i_cert[s]) == ref_idx
    print(f"shape {shape}: f64 re-decisions {tot_slow} of {5 * n_gen * per}")


# ------------------------------------------------------------------ physics
def test_physics_matches_oracle(gpu, oracle):
    from pong_amd.device import Physics
    rng = np.random.default_rng(3)
    n, steps = 384, 2500
    seeds = rng.integers(0, 2**62, size=n, dtype=np.int64)
    onep = (rng.random(n) < 0.3).astype(np.int32)
    ph = Physics(n, device=gpu)
    ph.reset(torch.tensor(seeds, device=gpu), torch.tensor(onep, device=gpu))
    envs = [oracle.Env(int(s), bool(o)) for s, o in zip(seeds, onep)]
    # actions: mostly paddle codes 0..2, occasionally both buttons
    acts = rng.integers(0, 16, size=(steps, n)).astype(np.uint8)
    names = ["ball_x", "ball_y", "ball_vx", "ball_vy", "ball_visible", "serve_timer", "serve_dir",
             "hits", "point", "lpy", "rpy", "score1", "score2"]
    for t in range(steps):
        ph.step(torch.tensor(acts[t], device=gpu))
        for i, e in enumerate(envs):
            a = int(acts[t, i])
            e.step4(a & 1, (a >> 1) & 1, (a >> 2) & 1, (a >> 3) & 1)
        if t % 50 == 49 or t == steps - 1:
            f = ph.fields()
            for name in names:
                got = f[name].numpy()
                want = np.array([getattr(e.state, name) for e in envs])
                np.testing.assert_array_equal(got, want, err_msg=f"field {name} at step {t}")


# --------------------------------------------------------------- episodes
def _schedule(rng, n, n_games, n_opp):
    kinds = np.zeros((n, n_games), np.int32)
    for g in range(n_games):
        kinds[:, g] = [0, 1, 2, 3, 3, 3][g % 6]
    flip = rng.random((n, n_games)) < 0.15
    kinds[flip] = 0  # empty-HoF style games
    opp = rng.integers(0, n_opp, size=(n, n_games)).astype(np.int32)
    mult = np.ones((n, n_games))
    hof_games = kinds == 3
    mult[hof_games] = np.round(rng.normal(size=hof_games.sum()), 3)
    return kinds, opp, mult


def _run_both(ev, oracle, genomes, opponents, kinds, opp, mult, gpu, **kw):
    dt = ev.dtype
    res, _ = ev.evaluate(_dev_genomes(genomes, gpu, dt), torch.tensor(kinds, device=gpu),
                         torch.tensor(opp, device=gpu), torch.tensor(mult, device=gpu),
                         opponents=_dev_genomes(opponents, gpu, dt), **kw)
    torch.cuda.synchronize()
    ref = oracle.eval_population(genomes, ev.nodes, kinds, opp, mult, opponents=opponents, bias=ev.bias,
                                 base_seed=ev.seed, n_threads=8)
    return res, ref


def _assert_same(res, ref):
    np.testing.assert_array_equal(res.scores.cpu().numpy(), ref["scores"])
    np.testing.assert_array_equal(res.frames.cpu().numpy(), ref["frames"])
    np.testing.assert_array_equal(res.total_frames.cpu().numpy(), ref["total_frames"])
    np.testing.assert_array_equal(res.rewards.cpu().numpy(), ref["rewards"])
    np.testing.assert_array_equal(res.fitness.cpu().numpy(), ref["fitness"])
    np.testing.assert_array_equal(res.status.cpu().numpy(), ref["status"])


@pytest.mark.parametrize("shape", SHAPES_RES + [[6, 8, 8, 3]])
@pytest.mark.parametrize("dist", ["init", "n3"])
def test_eval_matches_oracle(gpu, oracle, shape, dist):
    from pong_amd.device import Evaluator
    rng = np.random.default_rng(sum(shape) + (0 if dist == "init" else 7))
    G = _gene_count(shape)
    n, H = 97, 13  # ragged sizes on purpose
    draw = (lambda s: rng.random(s)) if dist == "init" else (lambda s: rng.standard_normal(s) * 3.0)
    genomes, opponents = draw((n, G)), draw((H, G))
    kinds, opp, mult = _schedule(rng, n, 6, H)
    ev = Evaluator(shape, device=gpu)
    res, ref = _run_both(ev, oracle, genomes, opponents, kinds, opp, mult, gpu)
    _assert_same(res, ref)
    # simulated env steps + periodic-rally frames not simulated = the episodes' frames
    assert int(res.counters[0]) + int(res.counters[8]) + int(res.counters[12]) == int(ref["frames"].sum())
    if len(shape) == 3:  # the other kernels must agree too
        for kernel, precision in (("general", "f64"),):
            res2, _ = ev.evaluate(_dev_genomes(genomes, gpu), torch.tensor(kinds, device=gpu),
                                  torch.tensor(opp, device=gpu), torch.tensor(mult, device=gpu),
                                  opponents=_dev_genomes(opponents, gpu), kernel=kernel, precision=precision)
            _assert_same(res2, ref)


@pytest.mark.parametrize("kernel,lanes,hidden", [
    ("split", 8, 4), ("split", 8, 8), ("split", 8, 64), ("split", 8, 37), ("split", 16, 16), ("split", 16, 64),
    ("split", 16, 40), ("split", 32, 64),
    ("split", 64, 64), ("split", 64, 256), ("split", 32, 50)])
def test_eval_kernel_layouts(gpu, oracle, kernel, lanes, hidden):
    """Every lane layout of the split kernel vs the oracle."""
    from pong_amd.device import Evaluator
    shape = [6, hidden, 3]
    rng = np.random.default_rng(lanes * 1000 + hidden)
    G = _gene_count(shape)
    genomes, opponents = rng.standard_normal((64, G)), rng.standard_normal((7, G))
    kinds, opp, mult = _schedule(rng, 64, 6, 7)
    ev = Evaluator(shape, device=gpu, group_lanes=lanes, kernel=kernel)
    res, ref = _run_both(ev, oracle, genomes, opponents, kinds, opp, mult, gpu)
    _assert_same(res, ref)


def test_eval_near_saturation_matches_oracle(gpu, oracle):
    """The bench distribution (N(0, 3) genes, [6,64,3], self-play): outputs sit
    near saturation, so the f32 certificate often fails and the service wave's
    plateau rule and memo decide; results must still equal the oracle's."""
    from pong_amd.device import Evaluator
    shape = [6, 64, 3]
    rng = np.random.default_rng(5)
    G = _gene_count(shape)
    n, H = 1536, 384
    genomes = rng.standard_normal((n, G)) * 3.0
    opponents = genomes[:H]
    kinds = np.full((n, 6), 3, np.int32)
    opp = ((np.arange(n)[:, None] * 6 + np.arange(6)[None, :]) % H).astype(np.int32)
    mult = np.ones((n, 6))
    ev = Evaluator(shape, device=gpu, kernel="split")
    res, ref = _run_both(ev, oracle, genomes, opponents, kinds, opp, mult, gpu)
    _assert_same(res, ref)
    c = res.counters.cpu().numpy()
    assert c[4] > 0 and c[5] > 0 and c[6] > 0, c    # in-wave and service certificates both exercised
    assert c[8] > 0, c                              # and periodic rallies skipped to their timeout
    assert c[2] + c[5] + c[6] <= c[4], c           # each failure is decided once


def test_eval_forward_count_by_frames(gpu, oracle):
    """The bench instance (8-lane groups, untraced) counts a game's forwards
    from its frame counter -- one hidden frame stepped per point, so visible
    frames = stepped frames - points -- while the other layouts count every
    visible frame: on a self-play launch the two agree with each other and
    with 2 x (stepped frames - points), and the results with the oracle."""
    from pong_amd.device import Evaluator
    shape = [6, 64, 3]
    rng = np.random.default_rng(17)
    G = _gene_count(shape)
    n, H = 384, 128
    genomes = rng.standard_normal((n, G)) * 3.0
    opponents = rng.standard_normal((H, G)) * 3.0
    kinds = np.full((n, 6), 3, np.int32)
    opp = rng.integers(0, H, size=(n, 6)).astype(np.int32)
    mult = np.ones((n, 6))
    counters = []
    for lanes in (8, 16):
        ev = Evaluator(shape, device=gpu, group_lanes=lanes, kernel="split")
        res, ref = _run_both(ev, oracle, genomes, opponents, kinds, opp, mult, gpu)
        _assert_same(res, ref)
        c = res.counters.cpu().numpy().astype(np.int64)
        points = int(res.scores.sum())
        assert c[1] == 2 * (c[0] - points), (lanes, c[0], c[1], points)
        counters.append(c)
    for i in (0, 1, 3, 8, 12):  # stepped frames, forwards, games, rally-skipped, hidden-jumped
        assert counters[0][i] == counters[1][i], (i, counters)


def test_eval_f32_genomes(gpu, oracle):
    """f32 genome storage: the oracle sees the same f32-rounded genes."""
    from pong_amd.device import Evaluator
    shape = [6, 64, 3]
    rng = np.random.default_rng(11)
    G = _gene_count(shape)
    genomes = rng.standard_normal((50, G)).astype(np.float32).astype(np.float64)
    opponents = rng.standard_normal((5, G)).astype(np.float32).astype(np.float64)
    kinds, opp, mult = _schedule(rng, 50, 6, 5)
    ev = Evaluator(shape, device=gpu, dtype=torch.float32)
    res, ref = _run_both(ev, oracle, genomes, opponents, kinds, opp, mult, gpu)
    _assert_same(res, ref)


def test_eval_edge_cases(gpu, oracle):
    from pong_amd.device import Evaluator
    shape = [6, 2, 2]
    ev = Evaluator(shape, device=gpu)
    G = _gene_count(shape)
    # empty population
    res, _ = ev.evaluate(torch.zeros((0, G), dtype=torch.float64, device=gpu),
                         torch.zeros((0, 6), dtype=torch.int32, device=gpu),
                         torch.zeros((0, 6), dtype=torch.int32, device=gpu),
                         torch.zeros((0, 6), dtype=torch.float64, device=gpu))
    assert res.fitness.numel() == 0
    # one genome, one game, padded rows (stride > gene count), all-zero weights (ties everywhere)
    ev1 = Evaluator(shape, device=gpu, n_games=1)
    g = torch.zeros((1, G + 5), dtype=torch.float64, device=gpu)
    res, _ = ev1.evaluate(g, torch.zeros((1, 1), dtype=torch.int32, device=gpu),
                          torch.zeros((1, 1), dtype=torch.int32, device=gpu),
                          torch.ones((1, 1), dtype=torch.float64, device=gpu))
    ref = oracle.eval_population(np.zeros((1, G)), shape, np.zeros((1, 1)), np.zeros((1, 1)), np.ones((1, 1)))
    np.testing.assert_array_equal(res.fitness.cpu().numpy(), ref["fitness"])
    np.testing.assert_array_equal(res.frames.cpu().numpy(), ref["frames"])
    # out-of-range opponent rows are refused on the host before launch
    with pytest.raises(ValueError):
        ev.evaluate(torch.zeros((1, G), dtype=torch.float64, device=gpu),
                    torch.full((1, 6), 3, dtype=torch.int32, device=gpu),
                    torch.full((1, 6), 5, dtype=torch.int32, device=gpu),
                    torch.ones((1, 6), dtype=torch.float64, device=gpu),
                    opponents=torch.zeros((2, G), dtype=torch.float64, device=gpu))


@pytest.mark.parametrize("name", ["episodes.json", "episodes_s3.json"])
@pytest.mark.parametrize("kernel", ["auto"])
def test_episode_traces_match_reference(gpu, golden, name, kernel):
    """Per-frame actions of the REAL perform_episode (tests/golden/episodes.json;
    episodes_s3.json: N(0, 3) genes, every game slot, long rallies and
    2 000-frame timeouts), traced; then untraced, where the kernels jump over
    periodic rallies -- frames, scores and rewards must not change."""
    from pong_amd.device import Evaluator
    eps = golden(name)
    for ep in eps:
        shape = ep["shape"]
        ev = Evaluator(shape, device=gpu, n_games=ep["game_index"] + 1, kernel=kernel)
        G = _gene_count(shape)
        n_games = ep["game_index"] + 1
        kinds = np.zeros((1, n_games), np.int32)
        kinds[0, ep["game_index"]] = ep["kind"]
        opp = np.zeros((1, n_games), np.int32)
        mult = np.ones((1, n_games))
        mult[0, ep["game_index"]] = ep["mult"]
        opponents = np.array([ep["opp"]]) if ep["opp"] is not None else np.zeros((1, G))
        cap = ep["frames"] + 1
        res, trace = ev.evaluate(_dev_genomes(np.array([ep["right"]]), gpu), torch.tensor(kinds, device=gpu),
                                 torch.tensor(opp, device=gpu), torch.tensor(mult, device=gpu),
                                 opponents=_dev_genomes(opponents, gpu), trace_games=n_games, trace_cap=cap)
        gi = ep["game_index"]
        assert int(res.frames[0, gi]) == ep["frames"]
        assert int(res.scores[0, gi, 0]) == ep["score1"] and int(res.scores[0, gi, 1]) == ep["score2"]
        assert float(res.rewards[0, gi]) == ep["reward"]
        tr = trace[gi, : ep["frames"]].cpu().numpy()
        # the action env.step received at frame t+1 is the decision traced at frame t
        np.testing.assert_array_equal(tr[:-1] & 3, np.array(ep["right_actions"][1:]))
        np.testing.assert_array_equal((tr[:-1] >> 2) & 3, np.array(ep["left_actions"][1:]))
        res2, _ = ev.evaluate(_dev_genomes(np.array([ep["right"]]), gpu), torch.tensor(kinds, device=gpu),
                              torch.tensor(opp, device=gpu), torch.tensor(mult, device=gpu),
                              opponents=_dev_genomes(opponents, gpu))
        assert int(res2.frames[0, gi]) == ep["frames"]
        assert int(res2.scores[0, gi, 0]) == ep["score1"] and int(res2.scores[0, gi, 1]) == ep["score2"]
        assert float(res2.rewards[0, gi]) == ep["reward"]


# ---------------------------------------------------------- full-size runs
def test_full_size_properties(gpu, oracle):
    """pop 65 536, [6,64,3] self-play: deterministic, permutation-equivariant,
    and a random sample of genomes re-checked against the oracle."""
    from pong_amd.device import Evaluator
    shape = [6, 64, 3]
    n, H = 65536, 16384
    G = _gene_count(shape)
    gen = torch.Generator(device=gpu).manual_seed(1234)
    genomes = torch.randn((n, G), generator=gen, dtype=torch.float64, device=gpu) * 3.0
    opponents = genomes[:H].contiguous()
    ev = Evaluator(shape, device=gpu)
    kind, opp, mult = ev.selfplay_schedule(n, H)
    r1, _ = ev.evaluate(genomes, kind, opp, mult, opponents=opponents)
    f1 = r1.fitness.clone()
    r2, _ = ev.evaluate(genomes, kind, opp, mult, opponents=opponents)
    assert torch.equal(f1, r2.fitness) and torch.equal(r1.frames, r2.frames)
    perm = torch.randperm(n, device=gpu)
    r3, _ = ev.evaluate(genomes[perm].contiguous(), kind[perm].contiguous(), opp[perm].contiguous(),
                        mult[perm].contiguous(), opponents=opponents)
    assert torch.equal(r3.fitness, f1[perm])
    assert int(r1.counters[3]) == n * 6 and int(r1.counters[0]) + int(r1.counters[8]) + int(r1.counters[12]) == int(r1.frames.sum())
    assert int(r1.counters[8]) > 0  # periodic rallies were jumped to their timeout
    sc = r1.scores.cpu().numpy()
    assert sc.max() <= 3 and sc.min() >= 0
    rng = np.random.default_rng(0)
    sel = rng.choice(n, size=48, replace=False)
    gsel = genomes[sel].cpu().numpy()
    ref = oracle.eval_population(gsel, shape, kind[sel].cpu().numpy(), opp[sel].cpu().numpy(),
                                 mult[sel].cpu().numpy(), opponents=opponents.cpu().numpy(), n_threads=8)
    np.testing.assert_array_equal(r1.fitness[sel].cpu().numpy(), ref["fitness"])
    np.testing.assert_array_equal(r1.frames[sel].cpu().numpy(), ref["frames"])


# ------------------------------------------------- fixed-horizon mode (8d)
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("T", [1, 37, 1000])
def test_horizon_matches_oracle(gpu, oracle, dtype, T):
    """pg_eval_args.horizon: every game slot runs exactly T frames with
    auto-reset; k_service (its horizon instance) equals the oracle's
    or_eval_population_h bit for bit (rewards summed over the completed
    episodes, every episode's points, completed-episode counts), in the
    saturation-heavy N(0, 3) distribution and over every game slot kind."""
    from pong_amd.device import Evaluator
    shape = [6, 64, 3]
    rng = np.random.default_rng(T + (0 if dtype == torch.float64 else 1))
    G = _gene_count(shape)
    n, H = 192, 48
    genomes = rng.standard_normal((n, G)) * 3.0
    opponents = rng.standard_normal((H, G)) * 3.0
    if dtype == torch.float32:
        genomes = genomes.astype(np.float32).astype(np.float64)
        opponents = opponents.astype(np.float32).astype(np.float64)
    kinds, opp, mult = _schedule(rng, n, 6, H)
    kinds[: n // 2] = 3  # half the population in all-network games
    ev = Evaluator(shape, device=gpu, dtype=dtype, horizon=T)
    res, _ = ev.evaluate(_dev_genomes(genomes, gpu, dtype), torch.tensor(kinds, device=gpu),
                         torch.tensor(opp, device=gpu), torch.tensor(mult, device=gpu),
                         opponents=_dev_genomes(opponents, gpu, dtype))
    torch.cuda.synchronize()
    ref = oracle.eval_population(genomes, shape, kinds, opp, mult, opponents=opponents, n_threads=8, horizon=T)
    _assert_same(res, ref)
    c = res.counters.cpu().numpy()
    assert c[0] == n * 6 * T and c[8] == 0 and c[12] == 0, c  # every frame stepped
    assert (res.frames.cpu().numpy() == T).all()
    if T == 1000:
        assert ref["total_frames"].sum() > n * 6  # multi-episode slots were exercised


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_horizon_long_slots_past_the_serve_table(gpu, oracle, dtype):
    """A horizon slot carries its point count across auto-resets; at T = 9000
    most slots pass kServeTabPoints = 64 points, where the serves stop coming
    from the block's LDS table and come from serve_entry(game_seed, point)
    (round-4 review: the tabbed slots had kept seed 0 there, so every slot got
    the same serves).  Bit-exact against the oracle, which serves every point
    from serve_entry(game_seed, point)."""
    from pong_amd.device import Evaluator
    shape = [6, 64, 3]
    T = 9000
    rng = np.random.default_rng(5)
    G = _gene_count(shape)
    n, H = 64, 16
    genomes = rng.standard_normal((n, G)) * 3.0
    opponents = rng.standard_normal((H, G)) * 3.0
    if dtype == torch.float32:
        genomes = genomes.astype(np.float32).astype(np.float64)
        opponents = opponents.astype(np.float32).astype(np.float64)
    kinds = np.tile(np.array([0, 1, 2, 3, 3, 3], np.int32), (n, 1))
    opp = rng.integers(0, H, (n, 6)).astype(np.int32)
    mult = np.where(kinds == 3, 0.5, 1.0)
    ev = Evaluator(shape, device=gpu, dtype=dtype, horizon=T)
    res, _ = ev.evaluate(_dev_genomes(genomes, gpu, dtype), torch.tensor(kinds, device=gpu),
                         torch.tensor(opp, device=gpu), torch.tensor(mult, device=gpu),
                         opponents=_dev_genomes(opponents, gpu, dtype))
    torch.cuda.synchronize()
    ref = oracle.eval_population(genomes, shape, kinds, opp, mult, opponents=opponents, n_threads=8, horizon=T)
    points = ref["scores"].sum(-1)
    assert (points > 64).sum() > n, "the regime past the serve table was not exercised"
    _assert_same(res, ref)
    assert (res.frames.cpu().numpy() == T).all()


def test_horizon_rejected_where_unsupported(gpu):
    from pong_amd import _lib
    from pong_amd.device import Evaluator
    shape = [6, 16, 3]
    G = _gene_count(shape)
    ev = Evaluator(shape, device=gpu, horizon=100)
    z = torch.zeros((4, 6), dtype=torch.int32, device=gpu)
    with pytest.raises(_lib.PongGAError):  # only the [6, 33..64, 3] layout has the horizon instance
        ev.evaluate(torch.zeros((4, G), dtype=torch.float64, device=gpu), z, z,
                    torch.ones((4, 6), dtype=torch.float64, device=gpu))
    ev = Evaluator([6, 64, 3], device=gpu, horizon=100)
    with pytest.raises(_lib.PongGAError):  # and it runs untraced
        ev.evaluate(torch.zeros((4, _gene_count([6, 64, 3])), dtype=torch.float64, device=gpu), z, z,
                    torch.ones((4, 6), dtype=torch.float64, device=gpu), trace_games=1, trace_cap=8)
