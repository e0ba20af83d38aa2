#!/usr/bin/env python3
"""Analysis (CPU, the oracle as the simulator): how long after the last point
do timeout games become periodic, and with what period?  Plays 1 500
self-play games of the bench distribution ([6,64,3], N(0,3) genes) with
traces, re-steps the timeout games and finds the first repeat of the full
rally state (pg_device.hpp rally_key's fields).  Measured: 55 timeouts, all
periodic with period 60, first repeat ~460 frames after the last point.
usage: python tools/rally_periods.py   (from the repository root)"""
import sys, numpy as np
sys.path.insert(0, 'oracle'); import oracle as O
rng = np.random.default_rng(0)
shape = [6, 64, 3]; G = 643
n = 1500
gen = rng.standard_normal((n, G)) * 3.0
H = 400
opp = gen[:H]
res = []
for i in range(n):
    g = i % 6
    j = (i * 6 + g) % H
    r = O.play_game(gen[i], shape, 3, opp[j], 1.0, O.game_seed(0, g), trace_cap=8192)
    if r["frames"] <= 2000: continue
    tr = r["trace"]
    env = O.Env(O.game_seed(0, g), False)
    seen = {}
    last_change = 0; prev_score = (0, 0); detect = None; period = None
    pv = None
    for t in range(1, r["frames"] + 1):
        a = tr[t - 2] if t >= 2 else 0
        rc, lc = a & 3, (a >> 2) & 3
        env.step4(rc == 1, rc == 2, lc == 1, lc == 2)
        s = env.snapshot()
        sc = (s["score1"], s["score2"])
        if sc != prev_score:
            seen = {}; last_change = t; prev_score = sc
        key = (s["ball_x"], s["ball_y"], s["ball_vx"], s["ball_vy"], s["ball_visible"], s["lpy"], s["rpy"],
               min(s["hits"], 8), s["serve_timer"], s["serve_dir"], pv, int(tr[t - 1]) & 15)
        pv = (s["ball_x"], s["ball_y"], s["ball_visible"])
        if key in seen and detect is None:
            detect = t; period = t - seen[key]
            break
        seen[key] = t
    res.append((r["frames"], last_change, detect, period))
res = np.array([(a, b, c if c else -1, d if d else -1) for a, b, c, d in res])
print("timeouts", len(res), "of", n)
print("frames", res[:, 0].mean(), "last change", res[:, 1].mean())
det = res[res[:, 2] > 0]
print("detected", len(det), "detect frame - last change: mean", (det[:, 2] - det[:, 1]).mean(), "max", (det[:, 2] - det[:, 1]).max(), "periods", np.percentile(det[:, 3], [50, 90, 100]))
print("saved frames per timeout game", (det[:, 0] - det[:, 2]).mean())
