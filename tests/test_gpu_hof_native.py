"""pg_hof_rank_classes (the device half of HallOfFame.update, one native
call) against the torch formulation DeviceGA otherwise uses (a stable sort in
age order + torch.unique), on the MI355X (-m gpu): identical ranks, the same
similarity partition as dense classes, the same fitness bits -- and the host
scan (pg_hof_update) returns the same hall from either packing.  Then whole
DeviceGA runs with and without it end with the same state."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _torch_packed(hf, hh, fc, h):
    old_n, k = hf.shape[0], fc.shape[0]
    n = old_n + k
    by_age = torch.cat([hf.flip(0), fc])
    order = torch.sort(by_age, stable=True).indices
    rank_age = torch.empty_like(order)
    rank_age[order] = torch.arange(n, device=fc.device)
    rank = torch.cat([rank_age[:old_n].flip(0), rank_age[old_n:]])
    cls = torch.unique(torch.cat([hh, h]), return_inverse=True)[1]
    return torch.cat([rank | (cls << 32), fc.view(torch.int64)])


@pytest.mark.parametrize("old_n,k", [(0, 1), (0, 300), (5, 1), (16, 3000), (1000, 10000), (16384, 2000),
                                     (131072, 25000)])
def test_rank_classes_match_torch_and_scan(gpu, old_n, k):
    from pong_amd import device as D
    rng = np.random.default_rng(old_n * 7 + k)
    # ties in fitness (rounded values) and duplicate hashes within and across the runs
    hf = np.sort(np.round(rng.standard_normal(old_n) * 3, 1))[::-1].copy()
    fc = np.round(rng.standard_normal(k) * 3 + 0.5, 1)
    hh = rng.permutation(np.unique(rng.integers(-2**63, 2**63 - 1, size=2 * old_n + 2, dtype=np.int64)))[:old_n]
    pool = rng.integers(-2**63, 2**63 - 1, size=max(8, k // 3), dtype=np.int64)
    h = pool[rng.integers(0, pool.size, k)]  # duplicates among the candidates
    if old_n:
        h[::5] = hh[rng.integers(0, old_n, h[::5].size)]  # and candidates similar to members
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)
    got = D.hof_rank_classes(t(hf), t(hh), t(fc), t(h)).cpu().numpy()
    ref = _torch_packed(t(hf), t(hh), t(fc), t(h)).cpu().numpy()
    n = old_n + k
    assert np.array_equal(got[:n] & 0xFFFFFFFF, ref[:n] & 0xFFFFFFFF), "ranks differ"
    assert np.array_equal(got[n:], ref[n:]), "fitness bits differ"
    cg, cr = got[:n] >> 32, ref[:n] >> 32
    allh = np.concatenate([hh, h])
    nu = np.unique(allh).size
    assert cg.min() >= 0 and cg.max() == nu - 1 and np.unique(cg).size == nu  # dense ids
    # same partition: class equality <=> hash equality (a bijection of labels)
    assert np.unique(np.stack([cg, allh]), axis=1).shape[1] == nu
    assert np.unique(np.stack([cr, allh]), axis=1).shape[1] == nu
    H = max(old_n, 1) if old_n else max(k // 4, 1)
    r1 = D.hof_update(H, hf, cg[:old_n], fc, cg[old_n:], rank=(got[:n] & 0xFFFFFFFF).astype(np.int32))
    r2 = D.hof_update(H, hf, cr[:old_n], fc, cr[old_n:], rank=(ref[:n] & 0xFFFFFFFF).astype(np.int32))
    assert np.array_equal(r1[0], r2[0]) and np.array_equal(r1[1], r2[1])


def test_rank_classes_rejects_short_workspace(gpu):
    import ctypes
    from pong_amd import _lib as L
    x = torch.zeros(4, dtype=torch.float64, device=gpu)
    hsh = torch.arange(4, dtype=torch.int64, device=gpu)
    out = torch.empty(12, dtype=torch.int64, device=gpu)
    a = L.PgHofRankArgs(4, x.data_ptr(), hsh.data_ptr(), 4, x.data_ptr(), hsh.data_ptr(), out.data_ptr(),
                        out.data_ptr(), 8)
    assert L.lib().pg_hof_rank_classes(ctypes.byref(a), None) != L.PG_OK


@pytest.mark.parametrize("pop", [64, 3000])
def test_device_ga_native_prepare_same_run(gpu, pop):
    from pong_amd.evolve import DeviceGA
    runs = []
    for native in (False, True):
        ga = DeviceGA([6, 8, 3], pop, device=gpu, schedule="selfplay", seed=99)
        ga.native_prepare = native
        ga.initialize("normal", 3.0)
        ga.run(4)
        runs.append((ga.hall_of_fame.clone(), ga.hof_member_fitness, ga.population.clone(), ga.fitness.clone(),
                     ga.logbook))
    a, b = runs
    assert torch.equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert torch.equal(a[2], b[2]) and torch.equal(a[3], b[3]) and a[4] == b[4]


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("pop,old_n,filtered", [(1, 0, False), (500, 0, False), (3000, 700, True),
                                                 (65536, 16384, True), (4000, 1000, True)])
def test_prepare_matches_torch_path(gpu, dtype, pop, old_n, filtered):
    """pg_hof_prepare = nonzero(fitness > worst) + pg_row_hash + the torch
    ranks/classes: same candidates, hashes and ranks, same partition."""
    from pong_amd import device as D
    rng = np.random.default_rng(pop + old_n)
    G = 37
    rows = torch.from_numpy(rng.standard_normal((pop, G))).to(gpu, dtype)
    rows[1::9] = rows[0]  # duplicate rows -> equal hashes
    fit = torch.from_numpy(np.round(rng.standard_normal(pop), 1)).to(gpu)
    hf = torch.from_numpy(np.sort(np.round(rng.standard_normal(old_n), 1))[::-1].copy()).to(gpu)
    hh = D.row_hash(torch.from_numpy(rng.standard_normal((max(old_n, 1), G))).to(gpu, dtype), G)[:old_n]
    if old_n > 3:
        hh[3] = D.row_hash(rows[:1], G)[0]  # a member similar to some candidates
    worst = float(hf[-1]) if filtered else None
    k, cand, hashes, packed = D.hof_prepare(fit, worst, rows, G, hf, hh)
    want = torch.nonzero(fit > worst).flatten() if filtered else torch.arange(pop, device=gpu)
    assert k == want.numel() and torch.equal(cand, want)
    if k == 0:
        return
    h = D.row_hash(rows, G, index=want.to(torch.int32))
    assert torch.equal(hashes, torch.cat([hh, h]))
    ref = _torch_packed(hf, hh, fit[want], h).cpu().numpy()
    got = packed.cpu().numpy()
    n = old_n + k
    assert np.array_equal(got[:n] & 0xFFFFFFFF, ref[:n] & 0xFFFFFFFF) and np.array_equal(got[n:], ref[n:])
    allh = hashes.cpu().numpy()
    nu = np.unique(allh).size
    assert np.unique(np.stack([got[:n] >> 32, allh]), axis=1).shape[1] == nu == np.unique(got[:n] >> 32).size
