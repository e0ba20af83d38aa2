"""Shared test setup.

* ``-m gpu`` tests need a real MI355X (they fail, never skip, without one).
* The oracle (oracle/) is imported here only as the checker.
"""
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "neuro-genetic-pong-self-play_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (os.path.join(REPO, "oracle"), PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def golden():
    def load(name):
        path = os.path.join(GOLDEN, name)
        if name.endswith(".json"):
            with open(path) as fh:
                return json.load(fh)
        if name.endswith(".npz"):
            return dict(np.load(path))
        return np.load(path)
    return load


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("this test needs a HIP device (run -m gpu on the MI355X box)")
    from pong_amd import build as B
    B.build()
    return torch.device("cuda", 0)

