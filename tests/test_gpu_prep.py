"""pg_eval_args.prep (ABI 7): the split kernel's lane records prepared in two
calls -- the genomes' before the hall of fame is known, the opponents' with
the games -- play exactly the games one call plays; the counters are zeroed
by the call itself (run with -m gpu)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(gpu, n, kernel, seed=3):
    from pong_amd.device import Evaluator
    ev = Evaluator([6, 64, 3], device=gpu, kernel=kernel)
    g = torch.Generator(device=gpu).manual_seed(seed)
    genomes = torch.randn((n + 17, ev.genes), generator=g, dtype=torch.float64, device=gpu) * 3.0
    hof = torch.randn((max(n // 4, 1), ev.genes), generator=g, dtype=torch.float64, device=gpu) * 3.0
    kind, opp, mult = ev.selfplay_schedule(n, hof.shape[0])
    rows = torch.randperm(n + 17, generator=g, device=gpu)[:n].to(torch.int32)
    count = torch.tensor([n - 5], dtype=torch.int32, device=gpu)
    return ev, genomes, hof, kind, opp, mult, rows, count


def _fields(res):
    return [res.fitness, res.rewards, res.scores, res.frames, res.total_frames, res.status, res.counters]


@pytest.mark.parametrize("kernel", ["split", "general"])
def test_prep_in_two_calls_equals_one(gpu, kernel):
    n = 600 if kernel == "split" else 24
    ev, genomes, hof, kind, opp, mult, rows, count = _setup(gpu, n, kernel)
    one, _ = ev.evaluate(genomes, kind, opp, mult, opponents=hof, rows=rows, n_active=count)
    one = [t.clone() for t in _fields(one)]
    out, _ = ev.evaluate(genomes, kind, opp, mult, opponents=hof, rows=rows, n_active=count)
    for t in _fields(out):
        t.fill_(7) if t.dtype != torch.float64 else t.fill_(-3.5)  # the counters too: the call zeroes them
    res, _ = ev.evaluate(genomes, kind, opp, mult, opponents=hof, rows=rows, n_active=count, out=out,
                         prep="genomes")
    assert all(torch.all(t == (7 if t.dtype != torch.float64 else -3.5)) for t in _fields(res))  # no games yet
    res, _ = ev.evaluate(genomes, kind, opp, mult, opponents=hof, rows=rows, n_active=count, out=out,
                         prep="rest")
    m = int(count[0])
    for a, b in zip(one, _fields(res)):
        if a.dim() >= 1 and a.shape[0] == n:
            assert torch.equal(a[:m], b[:m])  # entries >= n_active are left untouched
        else:
            assert torch.equal(a, b)
    assert int(res.counters[3]) == m * ev.n_games


def test_counters_zeroed_by_the_call(gpu):
    ev, genomes, hof, kind, opp, mult, rows, count = _setup(gpu, 256, "split", seed=5)
    genomes = genomes[:256]
    a, _ = ev.evaluate(genomes, kind, opp, mult, opponents=hof)
    first = a.counters.clone()
    a.counters.fill_(123456789)
    b, _ = ev.evaluate(genomes, kind, opp, mult, opponents=hof, out=a)
    assert torch.equal(first, b.counters)
