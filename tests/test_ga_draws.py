"""The numpy restatement of the device GA's counter-based draws (tests/_ga_draws.py)
against known answers; no GPU needed."""
import numpy as np

from _ga_draws import splitmix64, u01, rng_key, rng_u01, StubRandom


def test_splitmix64_known_answers():
    # SplitMix64's published first outputs for state 0 (x += golden gamma, then mix)
    assert int(splitmix64(0)) == 0xE220A8397B1DCDAF
    assert int(splitmix64(0x9E3779B97F4A7C15)) == 0x6E789E6AA1B965F4
    v = splitmix64(np.arange(4, dtype=np.uint64))
    assert [int(x) for x in v] == [int(splitmix64(i)) for i in range(4)]


def test_uniforms_in_range_and_keyed():
    a = u01(7, 3, 8, np.arange(1000), 0)
    assert a.min() >= 0.0 and a.max() < 1.0 and abs(a.mean() - 0.5) < 0.05
    assert not np.array_equal(a, u01(7, 4, 8, np.arange(1000), 0))
    k = rng_key(7, 3, 3, 5)
    g = rng_u01(k, np.arange(1000))
    assert g.min() >= 0.0 and g.max() < 1.0 and len(set(g.tolist())) == 1000


def test_stub_random_gauss_order():
    s = StubRandom([0.25, 0.5], [1.5])
    assert s.random() == 0.25 and s.gauss(1.0, 2.0) == 1.0 + 1.5 * 2.0 and s.random() == 0.5
