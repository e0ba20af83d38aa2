#!/usr/bin/env python3
"""Per-game wall-clock timeline of one pg_eval_population launch.

Needs a library built with -DPG_TIMELINE (PONG_GA_LIB=...): the split kernel
then writes {start, end, block, thread} (s_memrealtime, 100 MHz) per game into
the trace buffer instead of actions (and the block and wave that ran it).  Prints how the launch drains: games
still running over time, and when the longest games started.
usage: PONG_GA_LIB=variants/timeline.so python tools/timeline.py [--pop 65536] [--lanes 8]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "neuro-genetic-pong-self-play_amd"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--pop", type=int, default=65536)
    p.add_argument("--lanes", type=int, default=0)
    p.add_argument("--sigma", type=float, default=3.0)
    p.add_argument("--out", default="gpurun_out/timeline.npz")
    args = p.parse_args()
    import torch
    from pong_amd.device import Evaluator
    dev = torch.device("cuda", 0)
    n, H = args.pop, args.pop // 4
    ev = Evaluator([6, 64, 3], device=dev, group_lanes=args.lanes, kernel="split")
    gen = torch.Generator(device=dev).manual_seed(1234)
    genomes = torch.randn((n, ev.genes), generator=gen, dtype=torch.float64, device=dev) * args.sigma
    hof = genomes[:H].contiguous()
    kind, opp, mult = ev.selfplay_schedule(n, H)
    total = n * ev.n_games
    ev.evaluate(genomes, kind, opp, mult, opponents=hof)  # warm-up
    torch.cuda.synchronize()
    res, tr = ev.evaluate(genomes, kind, opp, mult, opponents=hof, trace_games=total, trace_cap=24)
    torch.cuda.synchronize()
    tl = tr.cpu().numpy().view(np.uint32).reshape(total, 6).astype(np.int64)
    frames = res.frames.cpu().numpy().reshape(-1)
    t0 = tl[:, 0].min()
    start = (tl[:, 0] - t0) / 100.0  # us
    end = (tl[:, 1] - t0) / 100.0
    span = end.max()
    out = {"pop": n, "games": total, "span_us": span}
    for q in (0.5, 0.9, 0.99, 0.999, 1.0):
        out[f"end_q{q}"] = float(np.quantile(end, q))
    long = frames > 1000
    out["long_games"] = int(long.sum())
    out["long_start_us_quantiles"] = [float(v) for v in np.quantile(start[long], [0, 0.5, 0.9, 0.99, 1.0])]
    dur = end - start
    out["us_per_frame_median"] = float(np.median(dur / np.maximum(frames, 1)))
    out["us_per_frame_long_median"] = float(np.median(dur[long] / frames[long]))
    last = np.argsort(end)[-5:]
    out["last_games"] = [{"frames": int(frames[i]), "start": float(start[i]), "end": float(end[i])} for i in last]
    fails, trips = tl[:, 2], tl[:, 3]
    out["fails_per_game_long_median"] = float(np.median(fails[long]))
    out["trips_per_frame_last"] = [float(trips[i] / max(frames[i], 1)) for i in last]
    # per-frame time vs service round trips per frame (games of > 500 frames)
    m = frames > 500
    if m.sum() > 10:
        A = np.stack([np.ones(m.sum()), trips[m] / frames[m]], 1)
        coef, *_ = np.linalg.lstsq(A, dur[m] / frames[m], rcond=None)
        out["fit_us_per_frame"] = float(coef[0])
        out["fit_us_per_trip"] = float(coef[1])
    # per game-wave index: frames per microsecond of wall time summed over each
    # wave's games (wave w runs on SIMD w % 4; the service wave shares SIMD 3)
    wave = tl[:, 5]
    out["frames_per_us_by_wave"] = {int(v): float(frames[wave == v].sum() / dur[wave == v].sum())
                                    for v in np.unique(wave)}
    out["us_per_frame_median_by_wave"] = {int(v): float(np.median(dur[wave == v] / np.maximum(frames[wave == v], 1)))
                                          for v in np.unique(wave)}
    grid = np.linspace(0, span, 21)
    out["running_games"] = [int(((start <= t) & (end > t)).sum()) for t in grid]
    print(json.dumps(out), flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    np.savez_compressed(args.out, start=start, end=end, frames=frames, fails=tl[:, 2], trips=tl[:, 3])


if __name__ == "__main__":
    main()
