"""Loader of tests/golden/nn_hard_cases.npz (tools/harvest_hard.py +
make_golden.py hard_cases): the decisions no bound settles, harvested on the
bench distribution, with the REAL reference's NeuralNetwork.run answers."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "nn_hard_cases.npz")


def load(label):
    """(shape, genes [n, G] f64 per case, x [n, 6], k [n, 6], idx_ref, act_ref, idx_device)."""
    h = dict(np.load(GOLDEN))
    shape = [int(v) for v in h[f"{label}__shape"]]
    seed, P, H, G, is64 = (int(v) for v in h[f"{label}__meta"])
    sigma = float(h[f"{label}__sigma"][0])
    dt = np.float64 if is64 else np.float32
    gen, is_opp, row, gidx = (h[f"{label}__{f}"] for f in ("gen", "is_opp", "row", "gidx"))
    need0 = (gen == 0).any()
    # generation-0 rows: the harvest drew them on the host from these seeds
    pop = (np.random.default_rng(seed).standard_normal((P, G)) * sigma).astype(dt) if need0 else None
    hof = (np.random.default_rng(seed + 1).standard_normal((H, G)) * sigma).astype(dt) if need0 else None
    stored = h[f"{label}__genes"]
    genes = np.stack([stored[gidx[i]] if gidx[i] >= 0 else (hof if is_opp[i] else pop)[row[i]]
                      for i in range(len(gen))]).astype(np.float64)
    k = h[f"{label}__k"].astype(np.int32)
    x = (k.astype(np.float64) / 2) / 160
    return dict(shape=shape, genes=genes, k=k, x=x, idx_ref=h[f"{label}__idx_ref"], act_ref=h[f"{label}__act_ref"],
                idx_device=h[f"{label}__idx_device"], total=h[f"{label}__total"])
