"""Diagnose pg_decide vs f64 argmax mismatches (test_decide_cascade_equals_f64)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "neuro-genetic-pong-self-play_amd"))
import numpy as np, torch
from pong_amd import build as B
B.build()
from pong_amd.device import Evaluator
gpu = torch.device("cuda", 0)
for shape in ([6, 200, 2], [6, 200, 3], [6, 128, 2], [6, 100, 2], [6, 64, 2], [6, 256, 2]):
    rng = np.random.default_rng(shape[1] * 7 + shape[2])
    G = sum((shape[i] + 1) * shape[i + 1] for i in range(len(shape) - 1))
    ev = Evaluator(shape, device=gpu)
    for sigma in (1.0, 3.0, 9.0, 30.0):
        n_gen, per = 512, 160
        gn = rng.standard_normal((n_gen, G)) * sigma
        genes = torch.tensor(gn, device=gpu)
        gi = np.repeat(np.arange(n_gen), per)
        k = rng.integers(0, 321, size=(n_gen * per, 6)).astype(np.int32)
        idx, stage = ev.decide(genes, torch.tensor(k, device=gpu), genome_index=torch.tensor(gi, dtype=torch.int32, device=gpu))
        x = torch.tensor(k * 0.5 / 160.0, device=gpu)
        ref, act = ev.forward(genes, x, genome_index=torch.tensor(gi, dtype=torch.int32, device=gpu), precision="f64", want_layers=True)
        idx, stage, ref = idx.cpu().numpy(), stage.cpu().numpy(), ref.cpu().numpy()
        z_all = ev.last_layers[0].cpu().numpy()
        bad = np.nonzero(idx != ref)[0]
        print(shape, sigma, "mismatch", len(bad), "stages", np.bincount(stage, minlength=4).tolist(), flush=True)
        for t in bad[:6]:
            print("   t", t, "dev", idx[t], "ref", ref[t], "stage", stage[t], "z_out", z_all[t, -shape[2]:].tolist(),
                  "act", act[t].cpu().numpy().tolist(), "k", k[t].tolist())
