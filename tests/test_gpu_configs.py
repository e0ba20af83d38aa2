"""BASELINE.json's GPU configs beyond the headline, each with an oracle re-play
(run with -m gpu):

* configs[1] -- population 4 096, MLP [6, 64, 3], one MI355X: the fused
  step + forward kernel (k_service) on a self-play evaluation against a
  1 024-row hall of fame, a sample of genomes re-played whole by the C oracle
  (main.py:28-66 evaluate, bit-exact), then the device-resident eaSimple
  (main.py:165-170) at that population: the initial evaluation and two
  generations, whose evaluations are re-played by the oracle as well;
* configs[4] -- the wide MLP [6, 512, 512, 3] at population 65 536 (k_wide, f32
  genome storage, a 16 384-row hall of fame): every game counted, a subset of
  the population evaluated on its own giving the same results (determinism and
  independence of the rows), and four genomes' evaluations re-played by the
  oracle (numpy_nn.py:120-137's f64 operation order, bit-exact)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _genes(shape):
    return sum((shape[i] + 1) * shape[i + 1] for i in range(len(shape) - 1))


def _replay(oracle, shape, genomes, kind, opp, mult, opponents, sel, res, n_threads=8):
    """The oracle's evaluate() of rows sel (each with the hall-of-fame rows its
    games use) against the device results res."""
    sel_t = torch.as_tensor(sel, device=genomes.device)
    rows = torch.unique(opp[sel_t].flatten())
    remap = torch.full((opponents.shape[0],), -1, dtype=torch.int32, device=genomes.device)
    remap[rows] = torch.arange(len(rows), dtype=torch.int32, device=genomes.device)
    ref = oracle.eval_population(genomes[sel_t].double().cpu().numpy(), shape, kind[sel_t].cpu().numpy(),
                                 remap[opp[sel_t].long()].cpu().numpy(), mult[sel_t].cpu().numpy(),
                                 opponents=opponents[rows].double().cpu().numpy(), n_threads=n_threads)
    for name in ("scores", "frames", "total_frames", "rewards", "fitness"):
        np.testing.assert_array_equal(getattr(res, name)[sel_t].cpu().numpy(), ref[name], err_msg=name)


def test_config2_pop4096_selfplay_against_oracle(gpu, oracle):
    from pong_amd.device import Evaluator
    shape = [6, 64, 3]
    G = _genes(shape)
    n, H = 4096, 1024
    gen = torch.Generator(device=gpu).manual_seed(4096)
    genomes = torch.randn((n, G), generator=gen, dtype=torch.float64, device=gpu) * 3.0
    opponents = torch.randn((H, G), generator=gen, dtype=torch.float64, device=gpu) * 3.0
    ev = Evaluator(shape, device=gpu)
    kind, opp, mult = ev.selfplay_schedule(n, H)
    res, _ = ev.evaluate(genomes, kind, opp, mult, opponents=opponents)
    torch.cuda.synchronize()
    c = res.counters.cpu().numpy()
    assert int(c[3]) == n * 6 and int(c[0]) + int(c[8]) + int(c[12]) == int(res.frames.sum())
    assert int(res.status.sum()) == 0 and bool(torch.isfinite(res.fitness).all())
    # 128 genomes re-played whole: a random sample plus the longest and the fittest
    rng = np.random.default_rng(2)
    sel = sorted(set(rng.choice(n, 126, replace=False).tolist())
                 | {int(res.frames.sum(dim=1).argmax()), int(res.fitness.argmax())})
    _replay(oracle, shape, genomes, kind, opp, mult, opponents, sel, res)


def test_config2_pop4096_device_ga_generations(gpu, oracle):
    """The device-resident eaSimple at population 4 096 (selection, variation,
    evaluation, hall of fame; bench.py's initialisation: a full hall of
    random genomes at fitness -1e300): every evaluation's sample of played
    rows re-played by the oracle through the on_evaluate hook."""
    from pong_amd.evolve import DeviceGA
    shape = [6, 64, 3]
    P = 4096
    ga = DeviceGA(shape, P, device=gpu, schedule="selfplay", seed=44)
    ga.initialize("normal", 3.0)
    H = ga.H
    ga.store[:H] = torch.randn((H, ga.G), generator=torch.Generator(device=gpu).manual_seed(45),
                               dtype=torch.float64, device=gpu) * 3.0
    ga.set_hall_of_fame(None, np.full(H, -1e300))
    checked = []

    def check(g, rows, opponents, res):
        n = res.fitness.shape[0]
        played = int(ga.last_count[0]) if ga.last_count is not None else n
        pick = np.unique(np.linspace(0, played - 1, 32).astype(np.int64))
        pt = torch.as_tensor(pick, device=gpu)
        r = ga.last_rows[pt].long() if ga.last_rows is not None else pt
        kind, opp, mult = ga.eval_schedule(g)
        o = opp[pt].cpu().numpy()
        used = np.unique(o)
        ref = oracle.eval_population(rows[r].double().cpu().numpy(), shape, kind[pt].cpu().numpy(),
                                     np.searchsorted(used, o).astype(np.int32), mult[pt].cpu().numpy(),
                                     opponents=opponents[torch.as_tensor(used, device=gpu)].double().cpu().numpy(),
                                     n_threads=8)
        np.testing.assert_array_equal(res.fitness[pt].cpu().numpy(), ref["fitness"])
        np.testing.assert_array_equal(res.frames[pt].cpu().numpy(), ref["frames"])
        checked.append(g)

    ga.on_evaluate = check
    ga.step()  # the initial evaluation
    ga.step()
    ga.step()
    assert len(checked) == 3
    assert len(ga.logbook) == 3 and all(np.isfinite(r["max"]) for r in ga.logbook)


def test_init_population_generations_every_row_against_oracle(gpu, oracle):
    """ga.py:85's initial genes, U[0, 1) -- the population every reference run
    starts from, whose evolved generations fail the f32 certificate on ~11 %
    of forwards (bench.py --dist init) and so drive the whole decision cascade
    (in-wave rules, the frame bound, the f64 stage, numpy's order): DeviceGA at
    population 4 096 against a full hall of U[0, 1) genomes, and every played
    row of the fourth evaluation re-played by the oracle, bit-exact; then 512
    of those rows and games in the fixed-horizon mode against the oracle's."""
    from pong_amd.evolve import DeviceGA
    shape = [6, 64, 3]
    P = 4096
    ga = DeviceGA(shape, P, device=gpu, schedule="selfplay", seed=46)
    ga.initialize("uniform")
    H = ga.H
    ga.store[:H] = torch.rand((H, ga.G), generator=torch.Generator(device=gpu).manual_seed(47),
                              dtype=torch.float64, device=gpu)
    ga.set_hall_of_fame(None, np.full(H, -1e300))
    seen = {}

    def keep(g, rows, opponents, res):
        n = res.fitness.shape[0]
        played = int(ga.last_count[0]) if ga.last_count is not None else n
        kind, opp, mult = ga.eval_schedule(g)
        pt = torch.arange(played, device=gpu)
        r = ga.last_rows[pt].long() if ga.last_rows is not None else pt
        seen[g] = dict(genomes=rows[r].double().cpu().numpy(), kind=kind[:played].cpu().numpy(),
                       opp=opp[:played].cpu().numpy(), mult=mult[:played].cpu().numpy(),
                       opponents=opponents.double().cpu().numpy(), fitness=res.fitness[:played].cpu().numpy(),
                       frames=res.frames[:played].cpu().numpy(), scores=res.scores[:played].cpu().numpy(),
                       counters=res.counters.cpu().numpy())

    ga.on_evaluate = keep
    for _ in range(4):  # the initial evaluation and three generations
        ga.step()
    g = max(seen)
    s = seen[g]
    c = s["counters"].astype(np.int64)
    assert c[4] > 0.05 * c[1], "expected the evolved U[0,1) population to fail the f32 certificate often"
    assert c[5] > 0, "expected decisions certified in f64"
    ref = oracle.eval_population(s["genomes"], shape, s["kind"], s["opp"], s["mult"], opponents=s["opponents"],
                                 n_threads=16)
    np.testing.assert_array_equal(s["fitness"], ref["fitness"])
    np.testing.assert_array_equal(s["frames"], ref["frames"])
    np.testing.assert_array_equal(s["scores"], ref["scores"])
    # the fixed-horizon instance (its own inline decision path) on the same
    # evolved genomes and games: 512 rows, T = 400 frames per slot, vs the oracle
    from pong_amd.device import Evaluator
    m, T = 512, 400
    ev = Evaluator(shape, device=gpu, horizon=T)
    opp_t = torch.tensor(s["opp"][:m], device=gpu)
    res_h, _ = ev.evaluate(torch.tensor(s["genomes"][:m], device=gpu), torch.tensor(s["kind"][:m], device=gpu),
                           opp_t, torch.tensor(s["mult"][:m], device=gpu),
                           opponents=torch.tensor(s["opponents"], device=gpu))
    torch.cuda.synchronize()
    ch = res_h.counters.cpu().numpy().astype(np.int64)
    assert ch[4] > 0.05 * ch[1], "expected the horizon instance to meet the population's certificate failures"
    ref_h = oracle.eval_population(s["genomes"][:m], shape, s["kind"][:m], s["opp"][:m], s["mult"][:m],
                                   opponents=s["opponents"], n_threads=16, horizon=T)
    for name in ("scores", "frames", "total_frames", "rewards", "fitness"):
        np.testing.assert_array_equal(getattr(res_h, name).cpu().numpy(), ref_h[name], err_msg=name)


def test_config5_wide_pop65536(gpu, oracle):
    from pong_amd.device import Evaluator
    shape = [6, 512, 512, 3]
    G = _genes(shape)
    n, H = 65536, 16384
    gen = torch.Generator(device=gpu).manual_seed(65536)
    genomes = torch.empty((n, G), dtype=torch.float32, device=gpu)
    for r0 in range(0, n, 8192):  # (generated in blocks: the f64 draw would need 140 GB at once)
        genomes[r0:r0 + 8192] = torch.randn((8192, G), generator=gen, dtype=torch.float32, device=gpu) * 3.0
    opponents = torch.randn((H, G), generator=gen, dtype=torch.float32, device=gpu) * 3.0
    ev = Evaluator(shape, dtype=torch.float32, device=gpu)
    kind, opp, mult = ev.selfplay_schedule(n, H)
    res, _ = ev.evaluate(genomes, kind, opp, mult, opponents=opponents)
    torch.cuda.synchronize()
    c = res.counters.cpu().numpy()
    assert int(c[3]) == n * 6 and int(c[0]) + int(c[8]) + int(c[12]) == int(res.frames.sum())
    assert int(c[7]) > 0  # network weight passes (each streams one network's genes)
    assert int(res.status.sum()) == 0 and bool(torch.isfinite(res.fitness).all())
    # determinism and independence: 512 rows evaluated on their own give the same results
    sub = torch.as_tensor(np.random.default_rng(5).choice(n, 512, replace=False), device=gpu)
    ev2 = Evaluator(shape, dtype=torch.float32, device=gpu)
    r2, _ = ev2.evaluate(genomes[sub].contiguous(), kind[sub].contiguous(), opp[sub].contiguous(),
                         mult[sub].contiguous(), opponents=opponents)
    torch.cuda.synchronize()
    for name in ("fitness", "frames", "scores", "rewards", "total_frames"):
        assert torch.equal(getattr(r2, name), getattr(res, name)[sub]), name
    # four genomes re-played by the oracle: the first, the last, the longest and the fittest
    pick = sorted({0, n - 1, int(res.frames.sum(dim=1).argmax()), int(res.fitness.argmax())})
    _replay(oracle, shape, genomes, kind, opp, mult, opponents, pick, res)
