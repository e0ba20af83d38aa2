"""The hard-decision fixture on the CPU: the oracle (np.dot's order, libm's
pow) against the REAL reference's answers, and the decisions the kernels made
when the cases were harvested (tools/harvest_hard.py on the MI355X).

The split cases are every forward the hot kernel's certified cascade could not
settle and handed to its numpy-order f64 forward (bench distribution: [6,64,3]
self-play, N(0, 3) genomes, 4 evaluations of 65 536 genomes); the wide cases
are k_wide decisions whose two largest activations lie within 1e-12."""
import numpy as np
import pytest

from _hard_cases import load


@pytest.mark.parametrize("label", ["split", "wide"])
def test_recorded_device_decisions_equal_reference(label):
    c = load(label)
    assert len(c["idx_ref"]) > 300
    np.testing.assert_array_equal(c["idx_device"], c["idx_ref"])


def test_oracle_on_hard_cases(oracle):
    for label, n_max in (("split", None), ("wide", 200)):
        c = load(label)
        n = len(c["idx_ref"]) if n_max is None else n_max
        for i in range(n):
            idx, act = oracle.nn_run(c["genes"][i], c["shape"], c["x"][i])
            assert idx == c["idx_ref"][i], (label, i)
            np.testing.assert_allclose(act, c["act_ref"][i], rtol=0, atol=1e-12)
