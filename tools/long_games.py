#!/usr/bin/env python3
"""How the longest games of a launch end (CPU replay with the oracle).

Reads the networks tools/timeline_ga.py saved for the launch's longest games,
replays each game with the C oracle (actions per frame) and its physics
(states per frame), and reports per no-score segment: its length, whether it
ended by the timeout, the first frame at which the rally state (rally_key's
fields + the frame's actions) repeats -- the earliest a periodic-rally jump
could fire -- its period, and the frame at which k_service's search (Brent's,
sampled at paddle bounces, pg_service.hpp) fires.

    python tools/long_games.py gpurun_out/r3_i2/tl12.npz [--games 50]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as O  # noqa: E402

RALLY_START, THRESH = 256, 2000


def replay(genes, opp_genes, kind, slot, seed, frames):
    g = O.play_game(genes, [6, 64, 3], int(kind), opp_genes, 1.0, O.game_seed(seed, int(slot)),
                    trace_cap=int(frames) + 8)
    tr = g["trace"]
    env = O.Env(O.game_seed(seed, int(slot)), False)
    env.reset()
    keys, score, hits = [], [], []
    ar = al = 0
    for f in range(len(tr)):
        env.step4(ar & 1, ar >> 1, al & 1, al >> 1)
        s = env.snapshot()
        ar, al = int(tr[f]) & 3, (int(tr[f]) >> 2) & 3
        keys.append((s["ball_x"], s["ball_y"], s["ball_vx"], s["ball_vy"], s["ball_visible"], s["serve_timer"],
                     s["serve_dir"], min(s["hits"], 8), s["point"], s["lpy"], s["rpy"], ar, al))
        score.append(s["score1"] + s["score2"])
        hits.append(s["hits"])
    return g, keys, score, hits


def segments(keys, score, hits, mode="hits"):
    # mode "hits": k_service since round 3 (open at a point's 8th return, first
    # span 64 frames); "timeout": the earlier rule (open at timeout 256, span 256)
    span0 = 64 if mode == "hits" else RALLY_START
    out = []
    timeout, seg0 = -1, 0
    at, saved, span, brent = -1, None, span0, None
    first, seen = None, {}
    for f in range(len(keys)):
        same = f == 0 or score[f] == score[f - 1]
        if not same:
            out.append(dict(start=seg0, end=f, first_repeat=first, brent=brent))
            seg0, at, brent, first, seen = f, -1, None, None, {}
        timeout = timeout + 1 if same else 0
        k = keys[f]
        if first is None:
            if k in seen:
                first = (seen[k] - seg0, f - seen[k])  # (frame of the first state of the cycle, period)
            else:
                seen[k] = f
        bounced = f > 0 and hits[f] != hits[f - 1]
        opens = hits[f] >= 8 if mode == "hits" else timeout >= RALLY_START
        if brent is None and bounced and opens and timeout <= THRESH:
            if at < 0 or at > timeout:
                saved, at, span = k, timeout, span0
            elif saved == k:
                brent = f - seg0
            elif timeout - at >= span:
                saved, at, span = k, timeout, 2 * span
    out.append(dict(start=seg0, end=len(keys), first_repeat=first, brent=brent))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--games", type=int, default=50)
    ap.add_argument("--mode", default="hits", choices=("hits", "timeout"))
    a = ap.parse_args()
    d = np.load(a.npz)
    seed = int(d["seed"][0])
    tot = dict(frames=0, stepped=0, ideal=0, timeout_segments=0, periodic=0, brent_hit=0)
    rows = []
    for i in range(min(a.games, len(d["top"]))):
        g, keys, score, hits = replay(d["top_genes"][i], d["top_opp_genes"][i], d["top_kind"][i], d["slot"][i],
                                      seed, d["top_frames"][i])
        assert g["frames"] == d["top_frames"][i], (g["frames"], d["top_frames"][i])
        segs = segments(keys, score, hits, a.mode)
        stepped = ideal = 0
        for s in segs:
            n = s["end"] - s["start"]
            to = n > THRESH  # a segment that ran into the timeout
            tot["timeout_segments"] += to
            if to and s["first_repeat"] is not None:
                tot["periodic"] += 1
                rep = s["first_repeat"][0] + s["first_repeat"][1]
                ideal += min(n, rep + 1)
            else:
                ideal += n
            if to and s["brent"] is not None:
                tot["brent_hit"] += 1
                stepped += s["brent"] + 1
            else:
                stepped += n
        tot["frames"] += len(keys)
        tot["stepped"] += stepped
        tot["ideal"] += ideal
        rows.append(dict(frames=len(keys), dur_us=float(d["top_dur"][i]), slot=int(d["slot"][i]), stepped=stepped,
                         ideal=ideal, segs=[(s["end"] - s["start"], s["first_repeat"], s["brent"]) for s in segs]))
    for r in rows[:20]:
        print(json.dumps(r))
    print(json.dumps(tot))


if __name__ == "__main__":
    main()
