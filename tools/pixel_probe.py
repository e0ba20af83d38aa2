#!/usr/bin/env python3
"""Time pg_render_frames and pg_find_stuff on n frames (HIP events) and print
the HBM rates: render writes 100 800 B per frame, find_stuff reads the
76 800 B crop.  usage: python tools/pixel_probe.py [n]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "neuro-genetic-pong-self-play_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pong_amd import device as D  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
dev = torch.device("cuda", 0)
ph = D.Physics(n, device=dev)
rng = np.random.default_rng(0)
ph.reset(torch.tensor(rng.integers(0, 2**62, size=n, dtype=np.int64), device=dev))
for _ in range(100):
    ph.step(torch.tensor(rng.integers(0, 16, size=n).astype(np.uint8), device=dev))
frames = D.render_frames(ph.state)
out = D.find_stuff(frames)
for name, fn, nbytes in (("render", lambda: D.render_frames(ph.state), 100800),
                         ("find_stuff", lambda: D.find_stuff(frames), 76800)):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    reps = 10
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"{name}: {n} frames {ms:.3f} ms/launch = {n * nbytes / (ms / 1e3) / 1e9:.0f} GB/s "
          f"({n / (ms / 1e3):.3e} frames/s)", flush=True)
