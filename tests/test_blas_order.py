"""numpy's np.dot(W, x) operation order, restated (oracle or_blas_dot) and
checked bit for bit against numpy on this host.

numpy_nn.run computes every layer as np.dot(w, column) (numpy_nn.py:127) with
w a C-contiguous float64 [out, in+1] matrix: numpy calls cblas_dgemv and
OpenBLAS runs dgemv_t.  Its summation order (4/2/1-output kernels, FMA or
not, 2048-element blocks, the m & 3 tail) is what "numpy's f64 result" means
at the ulp level; the oracle and the device's f64 paths follow it.  This pins
the restatement to the numpy that generated the golden fixtures (OpenBLAS
0.3.29, x86-64 AVX2/FMA kernel); on a host whose numpy uses another BLAS
kernel the order differs and the test is skipped."""
import numpy as np
import pytest


def _numpy_blas_is_openblas_x86():
    import platform
    if platform.machine() not in ("x86_64", "AMD64"):
        return False
    try:
        cfg = np.show_config(mode="dicts")
        blas = cfg["Build Dependencies"]["blas"]
        return "openblas" in blas.get("name", "").lower()
    except Exception:
        return False


pytestmark = pytest.mark.skipif(not _numpy_blas_is_openblas_x86(), reason="numpy is not on x86-64 OpenBLAS")

SHAPES = [(64, 7), (64, 6), (3, 65), (2, 65), (4, 65), (2, 7), (2, 3), (512, 7), (512, 513), (3, 513),
          (5, 9), (6, 7), (7, 7), (3, 10), (4, 2049), (3, 2051), (2, 4100), (9, 1), (5, 4)]


@pytest.mark.parametrize("shape", SHAPES)
def test_blas_gemv_matches_np_dot_bit_for_bit(oracle, shape):
    n, m = shape
    rng = np.random.default_rng(n * 10007 + m)
    trials = 40 if n * m < 20000 else 3
    for t in range(trials):
        scale = [1.0, 3.0, 30.0][t % 3]
        w = rng.standard_normal((n, m)) * scale
        x = rng.random(m) if t % 2 else rng.standard_normal(m)
        want = np.dot(w, x)
        got = oracle.blas_gemv(w, x)
        np.testing.assert_array_equal(got, want)


def test_sequential_sum_is_not_numpys_order(oracle):
    """The reason for the restatement: a left-to-right sum differs from np.dot."""
    rng = np.random.default_rng(1)
    w = rng.standard_normal((64, 7)) * 3
    x = rng.random(7)
    seq = np.array([sum(float(a) * float(b) for a, b in zip(row, x)) for row in w])  # noqa: E501 (0 + p0 + p1 ...)
    assert np.mean(seq != np.dot(w, x)) > 0.1
    np.testing.assert_array_equal(oracle.blas_gemv(w, x), np.dot(w, x))
