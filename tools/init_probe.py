#!/usr/bin/env python3
"""Classify the certificate failures that reach k_service's in-wave f64 stage
(serve_inline) on bench.py's --dist init workload (DeviceGA from U[0,1) genes,
ga.py:85): run with a library built with -DPG_INLINE_LOG
(tools/build_variant.py), which logs one record per request
{z0..z3, static bound e, frame bound, stage | idx << 8} into pg_eval_args.hard_log.

    PONG_GA_LIB=ab/log.so python tools/init_probe.py OUT.npz [generations=3] [uniform|normal]
    PONG_GA_LIB=ab/stages.so python tools/init_probe.py stages 3 uniform   (-DPG_SERVE_STAGES: cycles per stage)
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "neuro-genetic-pong-self-play_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pong_amd.evolve import DeviceGA  # noqa: E402


def stages(ga, dev):
    """PG_SERVE_STAGES build: one evaluation with hard_log as the stage accumulators."""
    ga.hard_log = torch.zeros((64, 8), dtype=torch.int32, device=dev)
    ga.step()
    acc = ga.hard_log.cpu().numpy().view(np.uint64).reshape(-1)
    names = ["plateau_decide (static e)", "frame bound (records + 64-lane sums)", "rules under the frame bound",
             "fast_f64_decide (genome + f64)", "numpy-order forward", "output layer reload wait"]
    for base, what in ((0, "first call"), (12, "the same request again (PG_SERVE_TWICE)")):
        if not acc[base + 6:base + 12].any():
            continue
        print(what)
        for i, nm in enumerate(names):
            n = int(acc[base + 6 + i])
            if n:
                print(f"  {nm:40s} calls {n:9d}  mean cycles {acc[base + i] / n:9.0f}  total {acc[base + i] / 1e9:7.2f} G")


def main(out, gens=3, dist="uniform"):
    dev = torch.device("cuda", 0)
    P = 65536
    ga = DeviceGA([6, 64, 3], P, P // 4, P // 4, device=dev, schedule="selfplay", seed=1234)
    ga.initialize(dist, 3.0)
    gen = torch.Generator(device=dev).manual_seed(1235)
    for r0 in range(0, ga.H, 4096):
        r1 = min(ga.H, r0 + 4096)
        blk = (torch.rand((r1 - r0, ga.G), generator=gen, dtype=torch.float64, device=dev) if dist == "uniform"
               else torch.randn((r1 - r0, ga.G), generator=gen, dtype=torch.float64, device=dev) * 3.0)
        ga.store[r0:r1] = blk
    ga.set_hall_of_fame(None, np.full(ga.H, -1e300))
    for _ in range(gens):
        ga.step()
    if out == "stages":
        return stages(ga, dev)
    cap = 1 << 21
    ga.hard_log = torch.zeros((cap, 8), dtype=torch.int32, device=dev)
    ga.step()
    c = ga.last.counters.cpu().numpy().astype(np.int64)
    n = min(int(c[9]), cap)
    rec = ga.hard_log[:n].cpu().numpy().view(np.uint32)
    z = rec[:, :4].view(np.float32)
    e, ef = rec[:, 4].view(np.float32), rec[:, 5].view(np.float32)
    stage, idx = rec[:, 6] & 255, (rec[:, 6] >> 8) & 255
    wave, net = rec[:, 6] >> 16, rec[:, 7]
    np.savez_compressed(out, z=z, e=e, ef=ef, stage=stage, idx=idx, wave=wave, net=net, counters=c)
    fwd = c[1]
    print(f"forwards {fwd}, certificate failures {c[4]} ({c[4] / fwd:.4f}), in-wave {c[6]}, f64-certified {c[5]}, "
          f"numpy-order {c[2]}, serve_inline requests {c[9]} ({c[9] / fwd:.5f} of forwards)")
    srt = np.sort(z[:, :3], axis=1)
    top1, top2 = srt[:, 2], srt[:, 1]
    for s, name in ((1, "plateau_decide (static e)"), (2, "frame bound rules"), (3, "fast_f64_decide"),
                    (4, "numpy-order forward")):
        m = stage == s
        if m.any():
            print(f"stage {s} {name}: {m.sum()}  top1 pct {np.percentile(top1[m], [5, 50, 95]).round(3)}  "
                  f"gap pct {np.percentile((top1 - top2)[m], [5, 50, 95])}  e med {np.median(e[m]):.3g}")
    # locality: of each wave's requests (log order is each wave's serving order),
    # how many repeat a network among that wave's last K requests -- what a
    # per-wave cache of the f64 genome values would hit
    for K in (1, 2, 4, 8):
        hits = tot = 0
        for wv in np.unique(wave):
            seq = net[wave == wv]
            for i in range(len(seq)):
                tot += 1
                hits += int(seq[i] in seq[max(0, i - K):i])
        print(f"requests repeating one of the wave's last {K} networks: {hits} of {tot} ({hits / max(tot, 1):.3f})")
    f3 = stage == 3
    for K in (1, 4):
        hits = tot = 0
        for wv in np.unique(wave[f3]):
            seq = net[f3 & (wave == wv)]
            for i in range(len(seq)):
                tot += 1
                hits += int(seq[i] in seq[max(0, i - K):i])
        print(f"f64-stage requests repeating one of the wave's last {K} f64-stage networks: {hits} of {tot} ({hits / max(tot, 1):.3f})")
    bands = [(-1e9, 0), (0, 22.2), (22.2, 30), (30, 36.7), (36.7, 1e9)]
    for lo, hi in bands:
        m = (top1 >= lo) & (top1 < hi)
        print(f"top1 in [{lo}, {hi}): {m.sum()}  top2 >= 36.7: {(m & (top2 >= 36.7)).sum()}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3, sys.argv[3] if len(sys.argv) > 3 else "uniform")
