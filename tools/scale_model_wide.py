#!/usr/bin/env python3
"""Strong-scaling model of BASELINE config 5 (wide MLP [6,512,512,3], pop
65 536 over N GPUs), measured on one GPU: the per-shard k_wide evaluation
times of N = 2, 4, 8 ranks, with contiguous shards (shard_range, each played
longest-lineage first) and with length-balanced shards (DeviceGA.balance_shards:
the whole population's rows ordered by the previous evaluation's longest game,
dealt to the ranks in snake order).  The generation's evaluation at N is the
slowest shard's (the fitness all-gather waits for it): straggler factor = max
shard / mean shard, efficiency of the evaluation = (one-GPU evaluation / N) /
max shard.

    python tools/scale_model_wide.py [generations=2] [P=65536]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "neuro-genetic-pong-self-play_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pong_amd import device as D  # noqa: E402
from pong_amd import dist as PD  # noqa: E402
from pong_amd.evolve import DeviceGA  # noqa: E402


def timed_eval(ga, rows_idx, hof):
    """One evaluation of the given population rows (in that order) against the
    hall (``hof``: its rows in items order): (ms by HIP events, stepped env-steps)."""
    dev = ga.device
    rows = torch.as_tensor(rows_idx, dtype=torch.int32, device=dev)
    kind, opp, mult = ga.eval_schedule(ga.generation + 1, rows=rows)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    res, _ = ga.ev.evaluate(ga._rows, kind, opp, mult, opponents=hof, validate=False, rows=rows)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b), int(res.counters[0].item())


def main(gens=2, P=65536):
    dev = torch.device("cuda", 0)
    ga = DeviceGA([6, 512, 512, 3], P, P // 4, P // 4, dtype=torch.float32, device=dev, schedule="selfplay", seed=1234)
    ga.initialize("normal", 3.0)
    gen = torch.Generator(device=dev).manual_seed(1235)
    for r0 in range(0, ga.H, 1024):
        r1 = min(ga.H, r0 + 1024)
        ga.store[r0:r1] = (torch.randn((r1 - r0, ga.G), generator=gen, dtype=torch.float64, device=dev) * 3.0).float()
    ga.set_hall_of_fame(None, np.full(ga.H, -1e300))
    for _ in range(gens):
        ga.step()
    lineage = ga.lineage_frames.cpu().numpy()
    # the whole population in one evaluation, longest lineage first (what one GPU plays)
    order = np.argsort(-lineage, kind="stable")
    hof = ga.hall_of_fame
    one_ms, one_steps = timed_eval(ga, order, hof)
    out = {"P": P, "generations": gens, "one_gpu_ms": one_ms, "one_gpu_steps": one_steps}
    print(json.dumps(out), flush=True)
    for N in (2, 4, 8):
        for mode in ("contiguous", "balanced"):
            ms, steps = [], []
            for r in range(N):
                if mode == "contiguous":
                    lo, hi = PD.shard_range(P, r, N)
                    idx = np.arange(lo, hi)
                    idx = idx[np.argsort(-lineage[lo:hi], kind="stable")]
                else:
                    pos = PD.deal_positions(-(-P // N), r, N).numpy()
                    idx = order[pos[pos < P]]
                m, s = timed_eval(ga, idx, hof)
                ms.append(m)
                steps.append(s)
            rec = {"N": N, "mode": mode, "shard_ms": ms, "shard_steps": steps, "max_ms": max(ms),
                   "mean_ms": float(np.mean(ms)), "straggler_factor": max(ms) / float(np.mean(ms)),
                   "eval_efficiency": one_ms / N / max(ms)}
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 2, int(sys.argv[2]) if len(sys.argv) > 2 else 65536)
