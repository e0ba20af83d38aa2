#!/usr/bin/env python3
"""Where the hall-of-fame update's wall time goes (host ops, syncs, device):
DeviceGA at the bench configuration, a few generations, then torch.profiler
over DeviceGA._hof_update for the next ones.
usage: python tools/diag/hof_trace.py [pop] [gens] > gpurun_out/hof_trace.txt"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "neuro-genetic-pong-self-play_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from torch.profiler import profile, record_function, ProfilerActivity  # noqa: E402

from pong_amd.evolve import DeviceGA  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
gens = int(sys.argv[2]) if len(sys.argv) > 2 else 4
dev = torch.device("cuda", 0)
ga = DeviceGA([6, 64, 3], P, device=dev, schedule="selfplay", seed=1234)
ga.initialize("normal", 3.0)
ga.store[: ga.H] = torch.randn((ga.H, ga.G), dtype=torch.float64, device=dev) * 3.0
ga.set_hall_of_fame(None, np.full(ga.H, -1e300))
ga.step()
for _ in range(4):
    ga.step()

orig = ga._hof_update
walls = []


def timed(*a, **k):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with record_function("HOF_UPDATE"):
        r = orig(*a, **k)
    torch.cuda.synchronize()
    walls.append((time.perf_counter() - t0) * 1e3)
    return r


ga._hof_update = timed
for _ in range(gens):
    ga.step()
print(f"hof_update wall (synced around it), {gens} gens: " + " ".join(f"{w:.3f}" for w in walls), flush=True)
walls.clear()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    for _ in range(gens):
        ga.step()
print(f"under the profiler: " + " ".join(f"{w:.3f}" for w in walls), flush=True)
print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=45, max_name_column_width=60), flush=True)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
prof.export_chrome_trace(os.path.join(REPO, "gpurun_out", f"hof_trace_{P}.json"))
