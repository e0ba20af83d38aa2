"""The generation's device work around the evaluation (csrc/pg_gen.hip,
DeviceGA.fused) against the torch formulation it replaces (run with -m gpu):
same populations, fitness and halls of fame generation by generation; each
entry point against a plain torch / numpy restatement of eaSimple's
bookkeeping (main.py:165-170, ga.py:89-94)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(fused, shape, P, H, schedule, dtype, gens, gpu, seed=21):
    from pong_amd.evolve import DeviceGA
    ga = DeviceGA(shape, P, hof_size=H, tournsize=max(P // 4, 1), dtype=dtype, device=gpu, schedule=schedule,
                  seed=seed)
    ga.fused = fused
    ga.initialize("normal", 3.0)
    for _ in range(gens):
        ga.step()
    return ga


@pytest.mark.parametrize("schedule,dtype,P,H", [("selfplay", torch.float64, 512, 128),
                                                ("reference", torch.float32, 300, 75),
                                                ("selfplay", torch.float64, 2048, 512)])
def test_fused_generation_equals_torch_path(gpu, schedule, dtype, P, H):
    a = _run(True, [6, 16, 3], P, H, schedule, dtype, 5, gpu)
    b = _run(False, [6, 16, 3], P, H, schedule, dtype, 5, gpu)
    assert torch.equal(a.population, b.population) and torch.equal(a.fitness, b.fitness)
    assert torch.equal(a.hall_of_fame, b.hall_of_fame)
    assert a.hof_member_fitness.tolist() == b.hof_member_fitness.tolist()
    assert torch.equal(a.hof_hash[: a.hof_n], b.hof_hash[: b.hof_n])
    assert torch.equal(a.hof_fitness[: a.hof_n], b.hof_fitness[: b.hof_n])
    for ra, rb in zip(a.logbook, b.logbook):
        assert ra["gen"] == rb["gen"] and ra["nevals"] == rb["nevals"]
        assert ra["min"] == rb["min"] and ra["max"] == rb["max"]
        assert ra["avg"] == pytest.approx(rb["avg"], rel=1e-12, abs=1e-300)
        assert ra["std"] == pytest.approx(rb["std"], rel=1e-9, abs=1e-300)
    assert torch.equal(a.lineage_frames, b.lineage_frames)


def test_merge_fitness_matches_numpy(gpu):
    from pong_amd import device as D
    rng = np.random.default_rng(4)
    ws = D.Workspaces(gpu)
    for n in (1, 7, 2048, 2049, 70001):
        fit = rng.standard_normal(n) * 3
        inh = rng.standard_normal(n)
        inv = (rng.random(n) < 0.8).astype(np.uint8)
        fit[rng.integers(0, n, size=min(n, 5))] = 1.5  # ties
        worst = 0.25
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(gpu)  # noqa: E731
        new = torch.empty(n, dtype=torch.float64, device=gpu)
        cand = torch.empty(n, dtype=torch.int32, device=gpu)
        cfit = torch.empty(n, dtype=torch.float64, device=gpu)
        summ = torch.empty(8, dtype=torch.float64, device=gpu)
        for filt in (None, worst):
            D.merge_fitness(t(fit), t(inv), t(inh), new, filt, cand, cfit, summ, ws)
            want = np.where(inv == 1, fit, inh)
            np.testing.assert_array_equal(new.cpu().numpy(), want)
            s = summ.cpu().numpy()
            assert s[0] == 0 and s[5] == inv.sum()
            assert s[1] == pytest.approx(want.mean(), rel=1e-12, abs=1e-12)
            assert s[2] == pytest.approx(want.std(), rel=1e-10)
            assert s[3] == want.min() and s[4] == want.max()
            idx = np.arange(n) if filt is None else np.nonzero(want > filt)[0]
            k = int(s[6])
            assert k == len(idx)
            np.testing.assert_array_equal(cand[:k].cpu().numpy(), idx)
            np.testing.assert_array_equal(cfit[:k].cpu().numpy(), want[idx])
        # NaN: flagged, excluded from the statistics and the candidates
        fit2 = fit.copy()
        fit2[n // 2] = np.nan
        inv2 = np.ones(n, np.uint8)
        D.merge_fitness(t(fit2), t(inv2), t(inh), new, None, cand, cfit, summ, ws)
        s = summ.cpu().numpy()
        assert s[0] == 1 and s[6] == n - 1
        if n > 1:
            assert s[4] == np.nanmax(fit2)


def test_order_matches_torch_argsort(gpu):
    from pong_amd import device as D
    rng = np.random.default_rng(6)
    ws = D.Workspaces(gpu)
    P, lo, n = 5000, 1200, 3000
    inv = torch.from_numpy((rng.random(P) < 0.7).astype(np.uint8)).to(gpu)
    lin = torch.from_numpy(rng.integers(0, 40, P).astype(np.float32) * 50).to(gpu)
    rows = torch.empty(n, dtype=torch.int32, device=gpu)
    count = torch.empty(1, dtype=torch.int32, device=gpu)
    for by_length in (True, False):
        D.order(n, lo, inv, lin, by_length, rows, count, ws)
        inv_s = inv[lo:lo + n].bool()
        key = torch.where(inv_s, lin[lo:lo + n] if by_length else torch.zeros_like(lin[lo:lo + n]),
                          torch.full_like(lin[lo:lo + n], -1.0))
        want = (torch.argsort(key, descending=True, stable=True) + lo).to(torch.int32)
        assert torch.equal(rows, want)
        assert int(count[0]) == int(inv_s.sum())


def test_select_ranked_equals_sorted_path(gpu):
    from pong_amd import device as D
    rng = np.random.default_rng(8)
    ws = D.Workspaces(gpu)
    for n in (3, 1000, 65536):
        fit = torch.from_numpy(np.round(rng.standard_normal(n), 2)).to(gpu)  # many ties
        a = D.select_ranked(fit, n, max(n // 4, 1), 5, 3, ws)
        b = D.select_tournament_ranked(fit, n, max(n // 4, 1), 5, 3)
        assert torch.equal(a, b)


def test_scatter_and_inherit(gpu):
    from pong_amd import device as D
    rng = np.random.default_rng(9)
    n, lo, games = 700, 100, 6
    perm = torch.from_numpy(rng.permutation(n).astype(np.int32) + lo).to(gpu)
    count = torch.tensor([500], dtype=torch.int32, device=gpu)
    res = D.EvalResult(fitness=torch.from_numpy(rng.standard_normal(n)).to(gpu),
                       rewards=None, scores=None,
                       frames=torch.from_numpy(rng.integers(1, 3000, (n, games)).astype(np.int32)).to(gpu),
                       total_frames=None, status=None, counters=None)
    shard = torch.empty(n, dtype=torch.float64, device=gpu)
    lineage = torch.full((lo + n,), 7.0, dtype=torch.float32, device=gpu)
    D.scatter_fitness(res, n, lo, perm, count, shard, lineage)
    want = torch.zeros(n, dtype=torch.float64, device=gpu)
    want[perm[:500].long() - lo] = res.fitness[:500]
    assert torch.equal(shard, want)
    lw = torch.full((lo + n,), 7.0, dtype=torch.float32, device=gpu)
    lw[perm[:500].long()] = res.frames[:500].max(dim=1).values.float()
    assert torch.equal(lineage, lw)
    chosen = torch.from_numpy(rng.integers(0, lo + n, 300).astype(np.int32)).to(gpu)
    inh = torch.empty(300, dtype=torch.float64, device=gpu)
    lo_out = torch.empty(300, dtype=torch.float32, device=gpu)
    fit_all = torch.from_numpy(rng.standard_normal(lo + n)).to(gpu)
    D.inherit(chosen, fit_all, inh, lineage, lo_out)
    assert torch.equal(inh, fit_all[chosen.long()]) and torch.equal(lo_out, lineage[chosen.long()])


@pytest.mark.parametrize("hn,k,dup", [(0, 50, False), (16, 40, True), (512, 3000, True), (4096, 100, False),
                                      (16384, 5000, True), (20000, 70000, False)])
def test_hof_prepare_cand_same_scan_as_rank_classes(gpu, hn, k, dup):
    """The candidate-only ranks and table classes feed pg_hof_update the same
    hall as pg_hof_rank_classes' full sorts (ties and duplicate rows included;
    the searches' LDS samples are exact up to 2 048 entries, sampled beyond:
    strides 2, 8 and 35 here)."""
    from pong_amd import device as D
    rng = np.random.default_rng(hn + k)
    G = 20
    rows = torch.from_numpy(rng.standard_normal((k + 10, G))).to(gpu)
    if dup:
        rows[5] = rows[2]
        rows[9] = rows[2]
    cand = torch.from_numpy(np.sort(rng.choice(k + 10, k, replace=False)).astype(np.int32)).to(gpu)
    cfit = torch.from_numpy(np.round(rng.standard_normal(k), 1) + 0.0).to(gpu)
    hof_rows = torch.from_numpy(rng.standard_normal((max(hn, 1), G))).to(gpu)[:hn]
    if dup and hn:
        hof_rows[hn // 2] = rows[2]  # a member similar to candidates
    hof_fit = torch.from_numpy(-np.sort(-np.round(rng.standard_normal(hn), 1)) + 0.0).to(gpu)
    hof_hash = D.row_hash(hof_rows, G) if hn else torch.zeros(0, dtype=torch.int64, device=gpu)
    ws = D.Workspaces(gpu)
    ch = torch.empty(k, dtype=torch.int64, device=gpu)
    packed = torch.empty(hn + 2 * k, dtype=torch.int64, device=gpu)
    D.hof_prepare_cand(hof_fit, hof_hash, cand, cfit, rows, G, ch, packed, ws)
    assert torch.equal(ch, D.row_hash(rows, G, index=cand))
    ref = D.hof_rank_classes(hof_fit, hof_hash, cfit, ch)
    a, b = packed.cpu().numpy(), ref.cpu().numpy()
    n = hn + k
    np.testing.assert_array_equal(a[:n] & 0xFFFFFFFF, b[:n] & 0xFFFFFFFF)  # ranks
    np.testing.assert_array_equal(a[n:], b[n:])                          # candidate fitness bits
    ca, cb = a[:n] >> 32, b[:n] >> 32                                     # same partition
    assert len(set(zip(ca.tolist(), cb.tolist()))) == len(set(ca.tolist())) == len(set(cb.tolist()))
    maxsize = max(hn, 8)
    hf = hof_fit.cpu().numpy()
    for cls in (ca, cb):
        got = D.hof_update(maxsize, hf, cls[:hn], a[n:].view(np.float64), cls[hn:], rank=(a[:n] & 0xFFFFFFFF))
        if cls is ca:
            first = got
        else:
            np.testing.assert_array_equal(first[0], got[0])
            np.testing.assert_array_equal(first[1], got[1])


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_vary_pair_mask_equals_full_vary(gpu, dtype):
    """pg_ga_args.pair_mask (sharded variation): a shard's pairs, then
    the pairs pg_ga_mark_pairs marks for scattered rows (outside the shard),
    written in two calls into one buffer, equal a full varAnd on those rows;
    unmarked rows are left as they were; the invalid flags are every row's."""
    from pong_amd import device as D
    P, G = 1001, 67
    g = torch.Generator(device=gpu).manual_seed(5)
    parents = torch.randn((P, G), generator=g, dtype=torch.float64, device=gpu).to(dtype)
    chosen = torch.randint(0, P, (P,), generator=g, device=gpu, dtype=torch.int32)
    kw = dict(cxpb=0.9, mutpb=0.9, alpha=0.9, mu=0.0, sigma=0.9, indpb=0.9, seed=3, generation=7)
    full, inv_full = D.vary(parents, chosen, G, **kw)
    pairs = (P + 1) // 2
    lo, hi = 333, 667  # the shard's rows: pairs [166, 334)
    skip = (lo >> 1, (hi + 1) >> 1)
    shard = torch.zeros(pairs, dtype=torch.uint8, device=gpu)
    shard[skip[0]:skip[1]] = 1
    out = torch.full((P, G), 7.0, dtype=dtype, device=gpu)
    _, inv = D.vary(parents, chosen, G, **kw, out=out, pair_mask=shard)
    assert torch.equal(inv, inv_full)
    rows = torch.tensor([0, 5, 400, 998, 1000, 5, -3, 1001, 2 * pairs + 7], dtype=torch.int32, device=gpu)
    more = torch.zeros(pairs, dtype=torch.uint8, device=gpu)
    D.mark_pairs(more, rows, skip=skip)
    excl = torch.zeros(pairs, dtype=torch.uint8, device=gpu)
    excl[499] = 1
    none = torch.zeros(pairs, dtype=torch.uint8, device=gpu)
    D.mark_pairs(none, rows, skip=skip, exclude=excl)
    assert none.nonzero().flatten().tolist() == [0, 2, 500]
    want = torch.zeros(pairs, dtype=torch.uint8)
    want[[0, 2, 499, 500]] = 1  # row 400's pair (200) is in the shard; -3, 1001 (pair 500 is row 1000's) ...
    assert more.cpu().tolist() == want.tolist()
    _, inv2 = D.vary(parents, chosen, G, **kw, out=out, pair_mask=more)
    assert torch.equal(inv2, inv_full)
    written = torch.zeros(P, dtype=torch.bool)
    for j in list(range(skip[0], skip[1])) + [0, 2, 499, 500]:
        written[2 * j: min(2 * j + 2, P)] = True
    w = written.to(gpu)
    assert torch.equal(out[w], full[w])
    assert bool((out[~w] == 7.0).all())


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_vary_pair_list_equals_mask(gpu, dtype):
    """pg_ga_args.pair_list (ABI 10): the marked pairs as pg_ga_list_pairs'
    compact list give the same rows (and those rows' invalid flags) as the
    mask, one wave per listed pair; other rows untouched."""
    from pong_amd import device as D
    P, G = 4001, 643
    g = torch.Generator(device=gpu).manual_seed(6)
    parents = torch.randn((P, G), generator=g, dtype=torch.float64, device=gpu).to(dtype)
    chosen = torch.randint(0, P, (P,), generator=g, device=gpu, dtype=torch.int32)
    kw = dict(cxpb=0.9, mutpb=0.9, alpha=0.9, mu=0.0, sigma=0.9, indpb=0.9, seed=4, generation=9)
    full, inv_full = D.vary(parents, chosen, G, **kw)
    pairs = (P + 1) // 2
    mask = torch.zeros(pairs, dtype=torch.uint8, device=gpu)
    rows = torch.randint(0, P, (300,), generator=g, device=gpu, dtype=torch.int32)
    D.mark_pairs(mask, rows)
    lst = torch.full((pairs,), -1, dtype=torch.int32, device=gpu)
    cnt = torch.zeros(1, dtype=torch.int32, device=gpu)
    D.list_pairs(mask, lst, cnt)
    marked = mask.nonzero().flatten()
    assert int(cnt.item()) == marked.numel()
    assert sorted(lst[: int(cnt.item())].tolist()) == marked.tolist()
    out = torch.full((P, G), 7.0, dtype=dtype, device=gpu)
    inv = torch.full((P,), 9, dtype=torch.uint8, device=gpu)
    D.vary(parents, chosen, G, **kw, out=out, invalid=inv, pair_list=(lst, cnt, rows.numel()))
    w = torch.zeros(P, dtype=torch.bool, device=gpu)
    for j in marked.tolist():
        w[2 * j: min(2 * j + 2, P)] = True
    assert torch.equal(out[w], full[w]) and bool((out[~w] == 7.0).all())
    assert torch.equal(inv[w], inv_full[w]) and bool((inv[~w] == 9).all())


@pytest.mark.parametrize("schedule,dtype,P,H,slices", [("selfplay", torch.float64, 2048, 512, 0),
                                                       ("reference", torch.float32, 600, 150, 0),
                                                       ("selfplay", torch.float64, 4096, 1024, 1024)])
def test_in_place_hall_equals_dense_commit(gpu, schedule, dtype, P, H, slices):
    """The hall kept in place (ABI 12: pg_hof_update_packed's slots,
    pg_hof_commit's dst_slot, the schedule's positions mapped to slots or a
    sliced hall's rows gathered) against the dense commit that rewrites the
    whole hall every generation: the same populations, fitness, halls, hashes
    and logbooks generation by generation."""
    from pong_amd.evolve import DeviceGA
    runs = []
    for in_place in (True, False):
        ga = DeviceGA([6, 16, 3], P, hof_size=H, tournsize=max(P // 4, 1), dtype=dtype, device=gpu,
                      schedule=schedule, seed=31, hof_block_rows=slices)
        ga.in_place_hall = in_place
        ga.initialize("normal", 3.0)
        halls = []
        for _ in range(6):
            ga.step()
            halls.append((ga.hall_of_fame.clone(), ga.hof_hash[: ga.hof_n].clone()))
        runs.append((ga, halls))
    (a, ha), (b, hb) = runs
    assert not a._slots_identity  # the slots did move
    for (ra, sa), (rb, sb) in zip(ha, hb):
        assert torch.equal(ra, rb) and torch.equal(sa, sb)
    assert torch.equal(a.population, b.population) and torch.equal(a.fitness, b.fitness)
    assert a.hof_member_fitness.tolist() == b.hof_member_fitness.tolist()
    assert a.logbook == b.logbook
    # the in-place hall's storage holds each member in its slot
    assert torch.equal(a._hall_buf[a.hof_slot[: a.hof_n].long()], b.hall_of_fame)
