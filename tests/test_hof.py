"""pg_hof_update (host C++ in libpong_ga.so, no GPU) against the DEAP
HallOfFame restatement (pong_amd.deap_compat.tools.HallOfFame, DEAP's
published algorithm; deap itself is absent offline, so parity is unpinned
beyond the restatement).  Individuals are one-gene lists whose gene is the
row hash, so DEAP's ``similar`` (operator.eq on the gene lists) is exactly
hash equality."""
import random

import numpy as np
import pytest

from pong_amd import device as D
from pong_amd.deap_compat import base, creator, tools


@pytest.fixture(scope="module")
def Ind():
    if not hasattr(creator, "HofFitness"):
        creator.create("HofFitness", base.Fitness, weights=(1.0,))
        creator.create("HofInd", list, fitness=creator.HofFitness)
    return creator.HofInd


def _mk(Ind, h, f):
    ind = Ind([int(h)])
    ind.fitness.values = (float(f),)
    return ind


def _ranks(keys_f, fit):
    """pg_hof_args.rank as DeviceGA._hof_update computes it: a stable sort in age order."""
    by_age = np.concatenate([np.asarray(keys_f, np.float64)[::-1], np.asarray(fit, np.float64)])
    order = np.argsort(by_age, kind="stable")
    rank_age = np.empty(order.size, np.int32)
    rank_age[order] = np.arange(order.size)
    n_old = len(keys_f)
    return np.concatenate([rank_age[:n_old][::-1], rank_age[n_old:]])


@pytest.mark.parametrize("given_rank", [False, True])
@pytest.mark.parametrize("seed", range(12))
def test_hof_update_matches_deap_restatement(Ind, seed, given_rank):
    rng = np.random.default_rng(seed)
    maxsize = int(rng.integers(1, 24))
    hof = tools.HallOfFame(maxsize)
    keys_f, keys_h = np.zeros(0), np.zeros(0, np.int64)
    for _ in range(6):  # successive generations
        n = int(rng.integers(0, 60))
        # few distinct fitness values (ties) and few distinct genes (duplicates)
        fit = rng.integers(0, 8, size=n).astype(np.float64) * 0.5
        hsh = rng.integers(-2**62, 2**62, size=8)[rng.integers(0, 8, size=n)]
        pop = [_mk(Ind, h, f) for h, f in zip(hsh, fit)]
        hof.update(pop)
        src, new_fit = D.hof_update(maxsize, keys_f, keys_h, fit, hsh,
                                    rank=_ranks(keys_f, fit) if given_rank else None)
        old_n = keys_f.shape[0]
        new_h = np.array([keys_h[s] if s < old_n else hsh[s - old_n] for s in src], dtype=np.int64)
        assert [i.fitness.values[0] for i in hof] == list(new_fit)
        assert [i[0] for i in hof] == list(new_h)
        keys_f, keys_h = new_fit, new_h


def test_hof_update_edge_cases(Ind):
    # empty population, maxsize 0, an empty hall taking population[0] first
    src, fit = D.hof_update(4, [], [], [], [])
    assert len(src) == 0
    src, fit = D.hof_update(0, [], [], [1.0, 2.0], [1, 2])
    assert len(src) == 0
    src, fit = D.hof_update(2, [], [], [1.0, 5.0, 5.0, 3.0], [7, 7, 8, 9])
    hof = tools.HallOfFame(2)
    hof.update([_mk(Ind, h, f) for h, f in zip([7, 7, 8, 9], [1.0, 5.0, 5.0, 3.0])])
    assert list(fit) == [i.fitness.values[0] for i in hof]
    assert list(src) == [2, 3]  # [8] at 5.0 then [9] at 3.0; [7] at 5.0 was similar to [7] at 1.0


def test_hof_update_rejects_bad_arguments():
    from pong_amd import _lib
    with pytest.raises(_lib.PongGAError):
        D.hof_update(1, [1.0, 2.0], [1, 2], [], [])  # more members than maxsize
    with pytest.raises(ValueError):
        D.hof_update(3, [1.0], [], [], [])
    with pytest.raises(_lib.PongGAError):
        D.hof_update(3, [1.0], [1], [2.0], [2], rank=[0, 2])  # rank out of range


def test_hof_update_large_is_fast():
    import time
    rng = np.random.default_rng(0)
    n, H = 65536, 16384
    t0 = time.perf_counter()
    src, fit = D.hof_update(H, [], [], rng.standard_normal(n), rng.integers(-2**62, 2**62, size=n))
    assert len(src) == H and np.all(np.diff(fit) <= 0)
    assert time.perf_counter() - t0 < 1.0
    random.seed(0)



@pytest.mark.parametrize("seed", range(40))
def test_hof_update_merge_path_larger(Ind, seed):
    """The merge path (members in items order, as DeviceGA always passes them)
    over larger halls and populations, full and filling, many ties and
    duplicates, against DEAP's HallOfFame."""
    rng = np.random.default_rng(1000 + seed)
    maxsize = int(rng.integers(1, 300))
    hof = tools.HallOfFame(maxsize)
    keys_f, keys_h = np.zeros(0), np.zeros(0, np.int64)
    genes = rng.integers(-2**62, 2**62, size=int(rng.integers(2, 400)))
    for _ in range(5):
        n = int(rng.integers(0, 600))
        fit = np.round(rng.standard_normal(n) * 2, int(rng.integers(0, 3)))
        hsh = genes[rng.integers(0, genes.size, size=n)]
        hof.update([_mk(Ind, h, f) for h, f in zip(hsh, fit)])
        src, new_fit = D.hof_update(maxsize, keys_f, keys_h, fit, hsh,
                                    rank=_ranks(keys_f, fit) if seed % 2 else None)
        old_n = keys_f.shape[0]
        new_h = np.array([keys_h[s] if s < old_n else hsh[s - old_n] for s in src], dtype=np.int64)
        assert [i.fitness.values[0] for i in hof] == list(new_fit)
        assert [i[0] for i in hof] == list(new_h)
        keys_f, keys_h = new_fit, new_h


def test_hof_update_general_path_unordered_members():
    """Members not in items order take the general (full rank bitmap) path:
    with distinct fitness the result equals the ordered call's, up to the
    members' permutation."""
    rng = np.random.default_rng(7)
    H = 64
    mf = rng.permutation(np.arange(H, dtype=np.float64))  # distinct, unordered
    mh = rng.integers(-2**62, 2**62, size=H)
    pf = rng.standard_normal(200) * 40 + 30
    ph = rng.integers(-2**62, 2**62, size=200)
    ph[::7] = mh[rng.integers(0, H, size=ph[::7].size)]  # some similar to members
    src_u, fit_u = D.hof_update(H, mf, mh, pf, ph)
    perm = np.argsort(-mf, kind="stable")  # items order
    src_o, fit_o = D.hof_update(H, mf[perm], mh[perm], pf, ph)
    assert list(fit_u) == list(fit_o)
    back = np.array([perm[s] if s < H else s for s in src_o])
    assert list(src_u) == list(back)


def _packing(keys_f, keys_h, fit, hsh):
    """pg_hof_prepare_cand's packing in numpy: ranks in ascending (fitness, age)
    order, dense classes (a member's: the first member of equal hash; a
    candidate's: that member, else hof_n + the first candidate of equal hash),
    then the candidates' fitness bits."""
    hn, k = len(keys_f), len(fit)
    rank = _ranks(keys_f, fit).astype(np.int64)
    first_m, cls = {}, np.empty(hn + k, np.int64)
    for e in range(hn):
        cls[e] = first_m.setdefault(int(keys_h[e]), e)
    first_c = {}
    for c in range(k):
        h = int(hsh[c])
        cls[hn + c] = first_m[h] if h in first_m else first_c.setdefault(h, hn + c)
    return np.concatenate([rank | (cls << 32), np.asarray(fit, np.float64).view(np.int64)])


@pytest.mark.parametrize("seed", range(40))
def test_hof_update_packed_matches_deap(Ind, seed):
    """pg_hof_update_packed (the O(k log k) scan DeviceGA uses) against DEAP's
    HallOfFame over successive generations: full and filling halls, ties,
    duplicates among candidates and with members."""
    rng = np.random.default_rng(2000 + seed)
    maxsize = int(rng.integers(1, 300))
    hof = tools.HallOfFame(maxsize)
    keys_f, keys_h = np.zeros(0), np.zeros(0, np.int64)
    genes = rng.integers(-2**62, 2**62, size=int(rng.integers(2, 400)))
    for _ in range(5):
        n = int(rng.integers(0, 600))
        fit = np.round(rng.standard_normal(n) * 2, int(rng.integers(0, 3)))
        hsh = genes[rng.integers(0, genes.size, size=n)]
        hof.update([_mk(Ind, h, f) for h, f in zip(hsh, fit)])
        src, new_fit = D.hof_update_packed(maxsize, keys_f, _packing(keys_f, keys_h, fit, hsh), n)
        old_n = keys_f.shape[0]
        new_h = np.array([keys_h[s] if s < old_n else hsh[s - old_n] for s in src], dtype=np.int64)
        assert [i.fitness.values[0] for i in hof] == list(new_fit)
        assert [i[0] for i in hof] == list(new_h)
        keys_f, keys_h = new_fit.copy(), new_h


def test_hof_update_packed_equals_general_large():
    """At BASELINE config 4's sizes (a 131 072-member hall, ~18 700 candidates
    above its worst) the packed scan returns pg_hof_update's result exactly."""
    rng = np.random.default_rng(9)
    H, k = 131072, 18721
    hof_f = np.sort(rng.normal(size=H))[::-1].copy()
    hof_h = rng.integers(-2**62, 2**62, size=H)
    fit = rng.normal(size=k) + 2.0
    hsh = rng.integers(-2**62, 2**62, size=k)
    hsh[::17] = hof_h[rng.integers(0, H, size=hsh[::17].size)]  # similar to members
    hsh[5::23] = hsh[rng.integers(0, k, size=hsh[5::23].size)]  # similar to other candidates
    packed = _packing(hof_f, hof_h, fit, hsh)
    src_p, fit_p = D.hof_update_packed(H, hof_f, packed, k)
    cls = packed[:H + k] >> 32
    src_g, fit_g = D.hof_update(H, hof_f, cls[:H], fit, cls[H:], rank=(packed[:H + k] & 0xFFFFFFFF).astype(np.int32))
    np.testing.assert_array_equal(src_p, src_g)
    np.testing.assert_array_equal(fit_p, fit_g)


def test_hof_update_packed_unordered_members_fall_back():
    rng = np.random.default_rng(3)
    H = 32
    mf = rng.permutation(np.arange(H, dtype=np.float64))
    mh = rng.integers(-2**62, 2**62, size=H)
    pf = rng.standard_normal(50) * 20 + 20
    ph = rng.integers(-2**62, 2**62, size=50)
    # ranks as the device would give them for these (unordered) members
    packed = _packing(mf, mh, pf, ph)
    src_p, fit_p = D.hof_update_packed(H, mf, packed, 50)
    cls = packed[:H + 50] >> 32
    src_g, fit_g = D.hof_update(H, mf, cls[:H], pf, cls[H:], rank=(packed[:H + 50] & 0xFFFFFFFF).astype(np.int32))
    np.testing.assert_array_equal(src_p, src_g)
    np.testing.assert_array_equal(fit_p, fit_g)


def _check_slots(old_slots, old_ids, src, slots, old_n):
    """The in-place hall's invariants: a storage array of ids (slot -> entry)
    updated by writing only the entering candidates holds member j's id in
    slot[j]; kept members kept their slots; the slots in use are [0, new_n)."""
    m = src.shape[0]
    store = np.full(max(m, old_n, 1), -1, np.int64)
    store[old_slots[:old_n]] = old_ids[:old_n]
    for j in range(m):
        if src[j] >= old_n:
            store[slots[j]] = 10**9 + src[j]  # a candidate's id
        else:
            assert slots[j] == old_slots[src[j]]  # a kept member stays in place
    ids = np.array([old_ids[s] if s < old_n else 10**9 + s for s in src], np.int64)
    np.testing.assert_array_equal(store[slots], ids)
    assert sorted(slots.tolist()) == list(range(m))
    return ids


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("unordered", [False, True])
def test_hof_update_packed_slots(seed, unordered):
    """pg_hof_update_packed's slot_out (ABI 12, the hall kept in place) over
    successive updates, on the packed scan and on its general fallback
    (unordered members): the same members as without slots, and a storage
    that receives only the entering candidates' rows holds every member in
    its slot."""
    rng = np.random.default_rng(7000 + seed)
    maxsize = int(rng.integers(1, 200))
    keys_f, keys_h = np.zeros(0), np.zeros(0, np.int64)
    slots, ids = np.zeros(0, np.int32), np.zeros(0, np.int64)
    genes = rng.integers(-2**62, 2**62, size=int(rng.integers(2, 300)))
    for gen in range(6):
        n = int(rng.integers(0, 400))
        fit = np.round(rng.standard_normal(n) * 2, int(rng.integers(0, 3)))
        hsh = genes[rng.integers(0, genes.size, size=n)]
        mf = keys_f
        if unordered and mf.shape[0] > 1:  # members out of items order: the general scan
            perm = rng.permutation(mf.shape[0])
            mf, keys_h, slots, ids = mf[perm], keys_h[perm], slots[perm], ids[perm]
        packed = _packing(mf, keys_h, fit, hsh)
        src0, fit0 = D.hof_update_packed(maxsize, mf, packed, n)
        src, new_fit, new_slots = D.hof_update_packed(maxsize, mf, packed, n, slot_in=slots, slots=True)
        np.testing.assert_array_equal(src, src0)
        np.testing.assert_array_equal(new_fit, fit0)
        old_n = mf.shape[0]
        ids = _check_slots(slots, ids, src, new_slots, old_n) + gen * 10**10 * (src >= old_n)
        keys_h = np.array([keys_h[s] if s < old_n else hsh[s - old_n] for s in src], dtype=np.int64)
        keys_f, slots = new_fit.copy(), new_slots.copy()


def test_hof_update_packed_slots_large_out_buffer():
    """Config 4's sizes with the outputs written into one upload buffer
    (fitness, sources, slots back to back), as DeviceGA passes it."""
    rng = np.random.default_rng(11)
    H, k = 131072, 18721
    hof_f = np.sort(rng.normal(size=H))[::-1].copy()
    hof_h = rng.integers(-2**62, 2**62, size=H)
    fit = rng.normal(size=k) + 2.0
    hsh = rng.integers(-2**62, 2**62, size=k)
    slots = rng.permutation(H).astype(np.int32)
    packed = _packing(hof_f, hof_h, fit, hsh)
    out = np.zeros(4 * H, np.int32)
    src, new_fit, new_slots = D.hof_update_packed(H, hof_f, packed, k, slot_in=slots, slots=True, out=out)
    src0, fit0 = D.hof_update_packed(H, hof_f, packed, k)
    np.testing.assert_array_equal(src, src0)
    np.testing.assert_array_equal(new_fit, fit0)
    np.testing.assert_array_equal(out[2 * H:2 * H + src.shape[0]], src)
    np.testing.assert_array_equal(out[:2 * H].view(np.float64)[:src.shape[0]], fit0)
    _check_slots(slots, np.arange(H, dtype=np.int64), src, new_slots, H)
    with pytest.raises(ValueError):
        D.hof_update_packed(H, hof_f, packed, k, out=np.zeros(4 * H - 1, np.int32))


def test_hof_update_packed_refuses_bad_slots():
    """slot_in outside [0, hof_n) is refused before any slot is handed out
    (the commit would write the hall's storage at those slots)."""
    rng = np.random.default_rng(5)
    H = 16
    hof_f = np.sort(rng.normal(size=H))[::-1].copy()
    hof_h = rng.integers(-2**62, 2**62, size=H)
    fit = rng.normal(size=4) + 3.0
    hsh = rng.integers(-2**62, 2**62, size=4)
    packed = _packing(hof_f, hof_h, fit, hsh)
    for bad in (-1, H):
        slots = np.arange(H, dtype=np.int32)
        slots[7] = bad
        with pytest.raises(RuntimeError):
            D.hof_update_packed(H, hof_f, packed, 4, slot_in=slots, slots=True)
