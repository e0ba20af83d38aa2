#!/usr/bin/env python3
"""Per-game timeline of the bench's own evaluation launch (after W GA
generations of bench.py's workload, length-ordered work queue).

Needs a -DPG_TIMELINE build (tools/build_variant.py timeline -DPG_TIMELINE):
the split kernel then writes {start, end, fails, trips, block, wave} per game
into the trace buffer.  Reports how the launch drains: games running over
time, the span after the queue empties, and the launch's tail cost against a
launch that kept every wave busy to the end.

    PONG_GA_LIB=variants/timeline.so python tools/timeline_ga.py [--gens 12]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "neuro-genetic-pong-self-play_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pop", type=int, default=65536)
    ap.add_argument("--gens", type=int, default=12)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--sigma", type=float, default=3.0)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "timeline_ga.npz"))
    ap.add_argument("--keep", type=int, default=200, help="longest games whose networks are saved")
    ap.add_argument("--no-order", action="store_true", help="evaluation order without the length prediction")
    args = ap.parse_args()
    import torch
    from pong_amd.evolve import DeviceGA
    dev = torch.device("cuda", 0)
    P, H = args.pop, args.pop // 4
    ga = DeviceGA([6, 64, 3], P, H, H, dtype=torch.float64, device=dev, n_games=6, schedule="selfplay",
                  seed=args.seed)
    ga.order_by_length = not args.no_order
    ga.initialize("normal", args.sigma)
    gen = torch.Generator(device=dev).manual_seed(args.seed + 1)
    ga.store[:H] = torch.randn((H, ga.G), generator=gen, dtype=torch.float64, device=dev).mul_(args.sigma)
    ga.set_hall_of_fame(None, np.full(H, -1e300))
    for _ in range(args.gens):
        ga.step()
    torch.cuda.synchronize(dev)

    captured = {}
    inner = ga.ev.evaluate

    def traced(*a, **kw):
        n_active = int(kw["n_active"].item()) if kw.get("n_active") is not None else a[0].shape[0]
        kw["trace_games"] = n_active * ga.ev.n_games
        kw["trace_cap"] = 24
        res, tr = inner(*a, **kw)
        captured["res"], captured["tr"], captured["n"] = res, tr, n_active
        captured["opp"] = a[2].clone()
        captured["kind"] = a[1].clone()
        captured["genomes"], captured["rows"] = a[0], kw.get("rows")
        captured["opponents"] = kw.get("opponents")
        return res, tr

    ga.ev.evaluate = traced
    ga.step()
    torch.cuda.synchronize(dev)
    ga.ev.evaluate = inner
    res, tr, n = captured["res"], captured["tr"], captured["n"]
    total = n * ga.ev.n_games
    tl = tr[:total].cpu().numpy().view(np.uint32).reshape(total, 6).astype(np.int64)
    frames = res.frames.cpu().numpy().reshape(-1)[:total]
    t0 = tl[:, 0].min()
    start = (tl[:, 0] - t0) / 100.0  # us (s_memrealtime, 100 MHz)
    end = (tl[:, 1] - t0) / 100.0
    span = float(end.max())
    queue_empty = float(start.max())  # the last game's start: the work counter ran out
    out = {"pop": P, "gens": args.gens, "ordered": not args.no_order, "games": total, "span_us": span,
           "queue_empty_us": queue_empty, "drain_us": span - queue_empty}
    for q in (0.5, 0.9, 0.99, 1.0):
        out[f"end_q{q}"] = float(np.quantile(end, q))
    grid = np.linspace(0, span, 41)
    running = np.array([int(((start <= t) & (end > t)).sum()) for t in grid])
    out["running_games"] = running.tolist()
    # busy game-slots integrated over time vs the full-occupancy plateau: the
    # fraction of the span the launch would save if every slot stayed busy
    fine = np.linspace(0, span, 2001)
    occ = np.array([((start <= t) & (end > t)).sum() for t in fine], dtype=np.float64)
    plateau = np.median(occ[(fine > 0.1 * span) & (fine < 0.5 * span)])
    out["plateau_games"] = float(plateau)
    out["occupancy_mean_frac"] = float(occ.mean() / plateau)
    out["tail_cost_frac"] = float(1.0 - occ.mean() / plateau)
    last = np.argsort(end)[-5:]
    out["last_games"] = [{"frames": int(frames[i]), "start": float(start[i]), "end": float(end[i])} for i in last]
    long = frames > 1000
    out["long_games"] = int(long.sum())
    if long.any():
        out["long_start_us_quantiles"] = [float(v) for v in np.quantile(start[long], [0, 0.5, 0.9, 1.0])]
    # what predicts a long game: the leave-one-out mean of the same genome's
    # other games, of the other games against the same opponent (this launch)
    opp = captured["opp"][:n].cpu().numpy().reshape(-1)[:total].astype(np.int64)
    dur = end - start
    gdur = dur.reshape(n, ga.ev.n_games)
    g_loo = (gdur.sum(1, keepdims=True) - gdur) / (ga.ev.n_games - 1)
    o_sum = np.bincount(opp, weights=dur, minlength=opp.max() + 1)
    o_cnt = np.bincount(opp, minlength=opp.max() + 1)
    o_loo = (o_sum[opp] - dur) / np.maximum(o_cnt[opp] - 1, 1)
    out["corr_dur_genome_loo"] = float(np.corrcoef(dur, g_loo.reshape(-1))[0, 1])
    out["corr_dur_opponent_loo"] = float(np.corrcoef(dur, o_loo)[0, 1])
    out["dur_us_quantiles"] = [float(v) for v in np.quantile(dur, [0.5, 0.9, 0.99, 0.999, 1.0])]
    print(json.dumps(out), flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    # the K longest games' networks, for a CPU replay of how they end (tools/long_games.py)
    top = np.argsort(-dur)[:args.keep]
    ent, slot = top // ga.ev.n_games, top % ga.ev.n_games
    rows = captured["rows"]
    grow = rows[torch.from_numpy(ent).to(dev)].long() if rows is not None else torch.from_numpy(ent).to(dev)
    keep = {"top": top, "slot": slot, "top_frames": frames[top], "top_dur": dur[top],
            "top_kind": captured["kind"].cpu().numpy().reshape(-1)[top],
            "top_genes": captured["genomes"][grow].double().cpu().numpy(),
            "top_opp_genes": captured["opponents"][torch.from_numpy(opp[top]).to(dev)].double().cpu().numpy(),
            "seed": np.array([ga.ev.seed], dtype=np.uint64)}
    np.savez_compressed(args.out, start=start, end=end, frames=frames, opp=opp, block=tl[:, 4], wave=tl[:, 5], **keep)


if __name__ == "__main__":
    main()
