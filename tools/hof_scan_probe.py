#!/usr/bin/env python3
"""What the host's hall-of-fame scan sees on the bench (diagnostic, GPU box):
runs bench.py's default command with pong_amd.device.hof_update_packed wrapped,
and prints per generation the candidate count k, the first output position
whose member changed (j0: [0, j0) is the old hall's prefix, unchanged) and the
wall time of the call (the C scan plus its numpy wrapper).

    python tools/hof_scan_probe.py [bench.py args ...]
"""
import os
import runpy
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "neuro-genetic-pong-self-play_amd"))
from pong_amd import device as D  # noqa: E402

_orig = D.hof_update_packed
rows = []


def wrapped(maxsize, hof_fitness, packed, k, slot_in=None, slots=False, out=None):
    t = time.perf_counter()
    res = _orig(maxsize, hof_fitness, packed, k, slot_in=slot_in, slots=slots, out=out)
    dt = time.perf_counter() - t
    src = res[0]
    hn = len(hof_fitness)
    changed = np.nonzero(src != np.arange(src.shape[0]))[0]
    j0 = int(changed[0]) if changed.size else int(src.shape[0])
    entering = int((src >= hn).sum())
    rows.append((int(k), hn, j0, entering, dt * 1e6))
    return res


D.hof_update_packed = wrapped
sys.argv = [os.path.join(REPO, "bench.py")] + (sys.argv[1:] or ["--steps", "20", "--warmup", "5", "--no-cpu-baseline"])
try:
    runpy.run_path(sys.argv[0], run_name="__main__")
finally:
    print("# gen  k  hof_n  j0  entering  scan_us", file=sys.stderr)
    for i, r in enumerate(rows):
        print("%3d %6d %6d %6d %6d %8.1f" % ((i,) + r), file=sys.stderr)
    if rows:
        a = np.array(rows, dtype=np.float64)
        print("# median k %.0f, j0 %.0f, entering %.0f, scan %.1f us" % tuple(np.median(a[:, c]) for c in (0, 2, 3, 4)),
              file=sys.stderr)
