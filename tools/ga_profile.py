#!/usr/bin/env python3
"""Per-phase wall time of DeviceGA.step() at the bench configuration
(pop 65 536, [6,64,3], self-play): select+vary, evaluate, hall of fame, record.
usage: python tools/ga_profile.py [pop] [steps]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "neuro-genetic-pong-self-play_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pong_amd.evolve import DeviceGA  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
dev = torch.device("cuda", 0)
ga = DeviceGA([6, 64, 3], P, device=dev, schedule="selfplay", seed=1234)
ga.initialize("normal", 3.0)
ga.store[: ga.H] = torch.randn((ga.H, ga.G), dtype=torch.float64, device=dev) * 3.0
ga.set_hall_of_fame(None, np.full(ga.H, -1e300))
ga.step()
for s in range(steps):
    ga.profile = {}
    t0 = time.perf_counter()
    rec = ga.step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    print(f"gen {rec['gen']}: {ms:.2f} ms  " + "  ".join(f"{k} {v:.2f}" for k, v in ga.profile.items())
          + f"  nevals {rec['nevals']} hof_n {ga.hof_n}", flush=True)

ga.profile = None
torch.cuda.synchronize()
t0 = time.perf_counter()
for s in range(steps):
    ga.step()
torch.cuda.synchronize()
print(f"unprofiled: {(time.perf_counter() - t0) * 1e3 / steps:.2f} ms per generation over {steps}", flush=True)
