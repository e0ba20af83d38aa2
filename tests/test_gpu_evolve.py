"""The device-resident eaSimple (pong_amd.evolve.DeviceGA) and its kernels:
pg_ga_schedule, pg_row_hash and the host pg_hof_update, on the MI355X
(run with -m gpu).

Parity: evaluations equal the C oracle's on the same schedule; the hall of
fame equals the DEAP HallOfFame restatement fed the same (fitness, gene-hash)
sequence; checkpoints resume bit for bit.  The GA's random draws are
counter-based (distribution parity with DEAP, not stream parity)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _gene_count(shape, bias=True):
    b = 1 if bias else 0
    return sum((shape[i] + b) * shape[i + 1] for i in range(len(shape) - 1))


def test_schedule_selfplay_equals_host(gpu):
    from pong_amd import device as D
    ev = D.Evaluator([6, 4, 3], device=gpu)
    for off in (0, 1000):
        k, o, m = D.schedule("selfplay", 77, 6, off, None, 13, 5, 2, gpu)
        k2, o2, m2 = ev.selfplay_schedule(77, 13, offset=off)
        assert torch.equal(k, k2) and torch.equal(o, o2) and torch.equal(m, m2)


@pytest.mark.parametrize("n_hof", [4096, 4099, 13])
def test_schedule_selfplay_sliced_hall(gpu, n_hof):
    """pg_schedule_args.hof_slices: row r of block b = r // B plays
    member k * K + b of the hall, k = (r * games + g) mod |slice b| -- or k
    itself with slice_local --, and a block evaluated against its slice alone
    equals the same rows evaluated against the whole hall (n_hof < K: the plain
    schedule)."""
    from pong_amd import device as D
    K, B, n, G6 = 4, 1000, 4000, 6
    rows = np.arange(n)
    k_, o, m = D.schedule("selfplay", n, G6, 0, None, n_hof, 5, 2, gpu, hof_slices=K, block_rows=B)
    o = o.cpu().numpy()
    if n_hof < K:
        want = (rows[:, None] * G6 + np.arange(G6)[None, :]) % n_hof
    else:
        b = (rows // B) % K
        msz = (n_hof - b + K - 1) // K
        kk = (rows[:, None] * G6 + np.arange(G6)[None, :]) % msz[:, None]
        want = kk * K + b[:, None]
    np.testing.assert_array_equal(o, want)
    if n_hof >= K:
        _, ol, _ = D.schedule("selfplay", n, G6, 0, None, n_hof, 5, 2, gpu, hof_slices=K, block_rows=B,
                              slice_local=True)
        np.testing.assert_array_equal(ol.cpu().numpy(), kk)
        # block 1's rows against slice 1 alone == against the whole hall
        shape = [6, 64, 3]
        G = _gene_count(shape)
        gen = torch.Generator(device=gpu).manual_seed(n_hof)
        genomes = torch.randn((B, G), generator=gen, dtype=torch.float64, device=gpu) * 3.0
        hall = torch.randn((n_hof, G), generator=gen, dtype=torch.float64, device=gpu) * 3.0
        ev = D.Evaluator(shape, device=gpu)
        kind = torch.full((B, G6), 3, dtype=torch.int32, device=gpu)
        mult = torch.ones((B, G6), dtype=torch.float64, device=gpu)
        r_full, _ = ev.evaluate(genomes, kind, torch.tensor(o[B:2 * B], device=gpu), mult, opponents=hall)
        ev2 = D.Evaluator(shape, device=gpu)
        r_slice, _ = ev2.evaluate(genomes, kind, torch.tensor(kk[B:2 * B].astype(np.int32), device=gpu), mult,
                                  opponents=hall[1::K])
        torch.cuda.synchronize()
        for name in ("fitness", "frames", "scores", "rewards"):
            assert torch.equal(getattr(r_full, name), getattr(r_slice, name)), name


def test_schedule_reference(gpu):
    from pong_amd import device as D
    n, H = 20000, 7
    hof_fit = torch.linspace(3.0, 1.0, H, dtype=torch.float64, device=gpu)
    k, o, m = D.schedule("reference", n, 6, 0, hof_fit, H, 11, 4, gpu)
    k, o, m = k.cpu().numpy(), o.cpu().numpy(), m.cpu().numpy()
    assert (k[:, :3] == [0, 1, 2]).all() and (k[:, 3:] == 3).all()   # main.py:39-53
    assert (m[:, :3] == 1.0).all()
    np.testing.assert_array_equal(m[:, 3:], hof_fit.cpu().numpy()[o[:, 3:]])
    counts = np.bincount(o[:, 3:].ravel(), minlength=H)
    exp = 3 * n / H
    assert ((counts - exp) ** 2 / exp).sum() < 30  # chi-square, 6 dof
    # deterministic per (seed, generation), different across generations
    k2, o2, _ = D.schedule("reference", n, 6, 0, hof_fit, H, 11, 4, gpu)
    assert np.array_equal(o, o2.cpu().numpy())
    _, o3, _ = D.schedule("reference", n, 6, 0, hof_fit, H, 11, 5, gpu)
    assert not np.array_equal(o, o3.cpu().numpy())
    # no hall of fame: HardcodedAi with multiplier 1 (main.py:44-45)
    k4, _, m4 = D.schedule("reference", 5, 6, 0, None, 0, 11, 4, gpu)
    assert (k4.cpu().numpy()[:, 3:] == 0).all() and (m4.cpu().numpy() == 1.0).all()


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_row_hash(gpu, dtype):
    from pong_amd import device as D
    g = torch.Generator(device=gpu).manual_seed(3)
    rows = torch.randn((50, 643), generator=g, device=gpu).to(dtype)
    rows[3, 10] = 0.0
    rows[7] = rows[3]
    rows[9] = rows[3]
    rows[9, 10] = -0.0  # list equality: 0.0 == -0.0
    rows[11] = rows[3]
    rows[11, 100] = torch.nextafter(rows[3, 100], torch.tensor(1e9, dtype=dtype, device=gpu))
    rows[20, :] = 0.0
    rows[21, :] = -0.0
    h = D.row_hash(rows).cpu().numpy()
    assert h[7] == h[3] and h[9] == h[3] and h[11] != h[3] and h[20] == h[21]
    assert len(set(h.tolist())) == 50 - 3
    idx = torch.tensor([11, 3, 49, 0], dtype=torch.int32, device=gpu)
    np.testing.assert_array_equal(D.row_hash(rows, index=idx).cpu().numpy(), h[[11, 3, 49, 0]])
    # hashing only the used genes of wider (padded) rows
    wide = torch.cat([rows, torch.randn((50, 5), generator=g, device=gpu).to(dtype)], dim=1)
    np.testing.assert_array_equal(D.row_hash(wide, genes=643).cpu().numpy(), h)


def _replay_hof(Ind, hof, ga, rows, fit):
    from pong_amd import device as D
    h = D.row_hash(rows, ga.G).cpu().numpy()
    inds = []
    for hv, f in zip(h, fit.cpu().numpy()):
        ind = Ind([int(hv)])
        ind.fitness.values = (float(f),)
        inds.append(ind)
    hof.update(inds)


@pytest.mark.parametrize("schedule,dtype", [("reference", torch.float64), ("selfplay", torch.float32)])
def test_device_ga_hall_of_fame_and_evaluations(gpu, oracle, schedule, dtype):
    """Every generation: the evaluated fitness equals the oracle's on the same
    schedule, and the hall of fame equals DEAP's HallOfFame.update replayed on
    the same (gene hash, fitness) sequence."""
    from pong_amd import device as D
    from pong_amd.deap_compat import base, creator, tools
    from pong_amd.evolve import DeviceGA
    if not hasattr(creator, "EvoFitness"):
        creator.create("EvoFitness", base.Fitness, weights=(1.0,))
        creator.create("EvoInd", list, fitness=creator.EvoFitness)
    shape = [6, 4, 3]
    ga = DeviceGA(shape, 96, hof_size=16, tournsize=8, dtype=dtype, device=gpu, schedule=schedule, seed=5)
    ga.initialize("normal", 2.0)
    hof = tools.HallOfFame(16)
    for step in range(4):
        g = ga.generation + 1
        hof_rows = ga.hall_of_fame.double().cpu().numpy()
        kind, opp, mult = D.schedule(schedule, ga.P, 6, 0, ga.hof_fitness, ga.hof_n, ga.seed, g, gpu)
        rec = ga.step()
        assert rec["gen"] == g
        # evaluations: recompute every offspring with the oracle on the same schedule
        pop = ga.population.double().cpu().numpy()
        ref = oracle.eval_population(pop, shape, kind.cpu().numpy(), opp.cpu().numpy(), mult.cpu().numpy(),
                                     opponents=hof_rows if len(hof_rows) else None, n_threads=8)
        fit = ga.fitness.cpu().numpy()
        # only eaSimple's invalid_ind are played (main.py:165-170); clones keep a parent's fitness
        m = ga.P if ga.last_count is None else int(ga.last_count[0])
        evaluated = ga.last.fitness[:m].cpu().numpy()
        rows_ev = np.arange(ga.P) if ga.last_rows is None else ga.last_rows[:m].cpu().numpy()
        assert len(rows_ev) == rec["nevals"] and rec["nevals"] > 0
        np.testing.assert_array_equal(evaluated, ref["fitness"][rows_ev])
        np.testing.assert_array_equal(fit[rows_ev], evaluated)
        _replay_hof(creator.EvoInd, hof, ga, ga.population, ga.fitness)
        assert [i.fitness.values[0] for i in hof] == ga.hof_member_fitness.tolist()
        hh = D.row_hash(ga.hall_of_fame, ga.G).cpu().numpy()
        assert [i[0] for i in hof] == hh.tolist()
    assert len(ga.logbook) == 4 and ga.logbook[-1]["max"] == float(ga.fitness.max())


def test_device_ga_checkpoint_resume(gpu, tmp_path):
    from pong_amd import checkpoint as C
    from pong_amd.evolve import DeviceGA
    kw = dict(hof_size=12, tournsize=6, device=gpu, schedule="reference", seed=9)
    a = DeviceGA([6, 3, 3], 64, **kw)
    a.initialize()
    a.run(3)
    b = DeviceGA([6, 3, 3], 64, **kw)
    b.initialize()
    b.run(1)
    path = C.save(b, str(tmp_path / "ga.safetensors"))
    c = C.load(path, device=gpu)
    c.step()
    c.step()
    assert torch.equal(a.population, c.population) and torch.equal(a.fitness, c.fitness)
    assert torch.equal(a.hall_of_fame, c.hall_of_fame)
    assert a.hof_member_fitness.tolist() == c.hof_member_fitness.tolist()
    assert a.logbook == c.logbook
    # the reference pickle round trip keeps population, fitness and hall of fame
    p = C.export_reference(c, str(tmp_path / "c_01_02_03.pkl"))
    d = C.import_reference(p, device=gpu, tournsize=6, schedule="reference", seed=9)
    assert torch.equal(d.population, c.population) and torch.equal(d.fitness, c.fitness)
    assert torch.equal(d.hall_of_fame, c.hall_of_fame) and bool(d.valid.all())
    rec = d.step()  # eaSimple's generation 0 of the resumed run: nothing to evaluate
    assert rec["nevals"] == 0 and torch.equal(d.fitness, c.fitness)


def test_longest_lineage_first_order(gpu):
    """DeviceGA plays a generation's invalid rows longest-lineage-first
    (order_by_length): the played rows come in non-increasing order of their
    lineage's longest game, clones after them, and the population, fitness,
    hall of fame and logbook equal those of the row-order run."""
    from pong_amd.evolve import DeviceGA
    kw = dict(hof_size=24, tournsize=12, device=gpu, schedule="selfplay", seed=13)
    runs, checked = {}, []
    for order in (True, False):
        ga = DeviceGA([6, 8, 3], 160, **kw)
        ga.order_by_length = order

        def probe(g, rows, opponents, res, ga=ga, order=order):
            # called before the evaluation's results update the predictions:
            # lineage_frames still holds the key the order was made with
            if order and ga.last_rows is not None:
                m = int(ga.last_count[0])
                key = ga.lineage_frames[ga.last_rows[:m].long()].cpu().numpy()
                assert (key[:-1] >= key[1:]).all(), key
                played = set(ga.last_rows[:m].cpu().tolist())
                assert len(played) == m
                checked.append(m)

        ga.on_evaluate = probe
        ga.initialize("normal", 3.0)
        for _ in range(4):
            ga.step()
        runs[order] = ga
    a, b = runs[True], runs[False]
    assert len(checked) == 4 and min(checked) > 0  # the initial evaluation and three generations
    assert torch.equal(a.population, b.population) and torch.equal(a.fitness, b.fitness)
    assert torch.equal(a.hall_of_fame, b.hall_of_fame)
    assert a.hof_member_fitness.tolist() == b.hof_member_fitness.tolist()
    assert a.logbook == b.logbook
    assert bool((a.lineage_frames > 0).any())
