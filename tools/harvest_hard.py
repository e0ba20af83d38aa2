#!/usr/bin/env python3
"""Harvest the decisions no bound settles, on the bench distribution.

Runs the bench's workload (DeviceGA, self-play vs the hall of fame, N(0, 3)
genomes, BASELINE config 3) for a few generations with pg_eval_args.hard_log
set: every forward the split kernel's service wave hands to the numpy-order
f64 forward is recorded as (network row, doubled-centroid features k, the
device's decision).  The same for the wide kernel ([6,512,512,3], sigma 3,
the initial evaluation): decisions whose two largest activations lie within
1e-12.

The initial population and hall of fame are drawn on the host
(numpy default_rng(seed) / (seed + 1), N(0, sigma)), so generation-0 rows are
regenerated from the seed wherever they are needed; rows of later generations
(varied on the device) are stored.  tests/golden/make_golden.py hard_cases
runs the real reference NeuralNetwork.run on every record (in the container)
and writes tests/golden/nn_hard_cases.npz; tests/test_gpu_hard_cases.py
replays it through pg_decide / pg_forward.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "neuro-genetic-pong-self-play_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def initial_rows(seed: int, n: int, G: int, sigma: float, dtype) -> np.ndarray:
    """The harvest's host-drawn rows: N(0, sigma), rounded to the storage dtype."""
    return (np.random.default_rng(seed).standard_normal((n, G)) * sigma).astype(dtype)


def harvest(shape, pop, gens, cap, sigma, seed, dtype, max_stored, dev, label):
    from pong_amd.evolve import DeviceGA
    P, H = pop, max(pop // 4, 1)
    npdt = np.float64 if dtype == torch.float64 else np.float32
    ga = DeviceGA(shape, P, H, H, dtype=dtype, device=dev, schedule="selfplay", seed=seed)
    G = ga.G
    ga.set_population(torch.from_numpy(initial_rows(seed, P, G, sigma, npdt)))
    ga.store[:H] = torch.from_numpy(initial_rows(seed + 1, H, G, sigma, npdt)).to(dev)
    ga.set_hall_of_fame(None, np.full(H, -1e300))
    ga.hard_log = torch.zeros((cap, 8), dtype=torch.int32, device=dev)
    cases, stored, total = [], {}, [0]
    forwards = [0]

    def hook(g, rows, opponents, res):
        cnt = int(res.counters[9])
        total[0] += cnt
        forwards[0] += int(res.counters[1])
        if cnt == 0:
            return
        recs = ga.hard_log[: min(cnt, cap)].cpu().numpy().view(np.uint32)
        for rec in recs:
            row, flags = int(rec[0]), int(rec[1])
            is_opp = flags & 1
            gidx = -1
            if g > 0:
                key = (g, is_opp, row)
                if key not in stored:
                    if len(stored) >= max_stored:
                        continue
                    src = opponents if is_opp else rows
                    stored[key] = (len(stored), src[row].cpu().numpy())
                gidx = stored[key][0]
            cases.append((g, is_opp, row, gidx, (flags >> 8) & 255, (flags >> 16) & 255, rec[2:8].astype(np.int32)))

    ga.on_evaluate = hook
    t0 = time.time()
    for _ in range(gens + 1):
        ga.step()
        print(f"[{label}] gen {ga.generation}: {total[0]} hard decisions of {forwards[0]} forwards, "
              f"{len(cases)} kept ({time.time() - t0:.1f} s)", flush=True)
    genes = [v[1] for v in sorted(stored.values(), key=lambda t: t[0])]
    return {
        f"{label}__shape": np.array(shape, np.int32),
        f"{label}__meta": np.array([seed, P, H, G, 1 if dtype == torch.float64 else 0], np.int64),
        f"{label}__sigma": np.array([sigma]),
        f"{label}__gen": np.array([c[0] for c in cases], np.int32),
        f"{label}__is_opp": np.array([c[1] for c in cases], np.int32),
        f"{label}__row": np.array([c[2] for c in cases], np.int32),
        f"{label}__gidx": np.array([c[3] for c in cases], np.int32),
        f"{label}__idx_device": np.array([c[4] for c in cases], np.int32),
        f"{label}__k": np.stack([c[6] for c in cases]) if cases else np.zeros((0, 6), np.int32),
        f"{label}__genes": np.stack(genes) if genes else np.zeros((0, G), npdt),
        f"{label}__total": np.array([total[0], forwards[0]], np.int64),
    }


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--pop", type=int, default=65536)
    p.add_argument("--gens", type=int, default=3)
    p.add_argument("--cap", type=int, default=1 << 16)
    p.add_argument("--max-stored", type=int, default=200, help="rows of generations >= 1 kept (5 KB each)")
    p.add_argument("--wide-pop", type=int, default=512)
    p.add_argument("--sigma", type=float, default=3.0)
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--out", default="gpurun_out/hard/hard_cases.npz")
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    from pong_amd import build as B
    B.build()
    out = harvest([6, 64, 3], a.pop, a.gens, a.cap, a.sigma, a.seed, torch.float64, a.max_stored, dev, "split")
    if a.wide_pop > 0:  # the initial evaluation only: every row regenerates from the seed
        out.update(harvest([6, 512, 512, 3], a.wide_pop, 0, a.cap, a.sigma, a.seed, torch.float32, 0, dev, "wide"))
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    np.savez_compressed(a.out, **out)
    print("wrote", a.out, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
