"""The device GA's counter-based draws restated in numpy (test infrastructure):
splitmix64 and the keys of k_select / k_select_ranked / k_vary
(csrc/pong_ga.hip u01, rng_key, rng_u01), so a test can recompute, from the
same draws, what DEAP's operators (ga.py:89-94: cxBlend, mutGaussian,
selTournament) give and compare the device's offspring bit for bit."""
import numpy as np

M64 = (1 << 64) - 1
C_GOLDEN = 0x9E3779B97F4A7C15
C_STREAM = 0xD6E8FEB86659FD93


def splitmix64(x):
    """Vectorised splitmix64 on uint64 arrays (or Python ints)."""
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x + np.uint64(C_GOLDEN)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def _gen_key(seed, gen):
    return int(splitmix64((seed + C_GOLDEN * (gen + 1)) & M64))


def u01(seed, gen, stream, a, b):
    """u01(seed, generation, stream, a, b) of pong_ga.hip (k_select / k_select_ranked)."""
    with np.errstate(over="ignore"):
        k = splitmix64(np.uint64(_gen_key(seed, gen)) ^ ((np.uint64(stream) * np.uint64(C_STREAM)) + np.asarray(a, np.uint64)))
    k = splitmix64(k ^ np.asarray(b, np.uint64))
    return (k >> np.uint64(11)).astype(np.float64) * 2.0 ** -53


def rng_key(seed, gen, stream, a):
    """rng_key(seed, generation, stream, a) of pong_ga.hip (k_vary)."""
    with np.errstate(over="ignore"):
        return splitmix64(np.uint64(_gen_key(seed, gen)) ^ ((np.uint64(stream) * np.uint64(C_STREAM)) + np.asarray(a, np.uint64)))


def rng_u01(key, b):
    return (splitmix64(np.asarray(key, np.uint64) ^ np.asarray(b, np.uint64)) >> np.uint64(11)).astype(np.float64) * 2.0 ** -53


class StubRandom:
    """Stands in for the ``random`` module inside deap_compat.tools: random()
    and gauss() hand out prepared draws in call order."""

    def __init__(self, uniforms=(), normals=()):
        self.u = list(uniforms)
        self.z = list(normals)
        self.iu = self.iz = 0

    def random(self):
        v = self.u[self.iu]
        self.iu += 1
        return float(v)

    def gauss(self, mu, sigma):  # random.gauss: mu + z * sigma
        z = self.z[self.iz]
        self.iz += 1
        return mu + float(z) * sigma
