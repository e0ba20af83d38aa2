#!/usr/bin/env python3
"""Host-side cost of the bench's generation: cProfile over DeviceGA.step() at
the bench's workload (population 65 536, [6,64,3], self-play against a full
hall of fame), after warm-up; the device's work overlaps it, so this is the
host's share of the time between two evaluations.

    python tools/host_profile.py [generations=20] > profile.txt
"""
import cProfile
import io
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "neuro-genetic-pong-self-play_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pong_amd.evolve import DeviceGA  # noqa: E402


def main(gens=20):
    dev = torch.device("cuda", 0)
    P = 65536
    ga = DeviceGA([6, 64, 3], P, P // 4, P // 4, device=dev, schedule="selfplay", seed=1234, hof_block_rows=P)
    ga.initialize("normal", 3.0)
    g = torch.Generator(device=dev).manual_seed(1235)
    ga.store[:ga.H] = torch.randn((ga.H, ga.G), generator=g, dtype=torch.float64, device=dev) * 3.0
    ga.set_hall_of_fame(None, np.full(ga.H, -1e300))
    for _ in range(5):
        ga.step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(gens):
        ga.step()
    pr.disable()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3 / gens
    s = io.StringIO()
    st = pstats.Stats(pr, stream=s).sort_stats("tottime")
    st.print_stats(35)
    print(f"# {gens} generations, {wall:.3f} ms each (wall, under cProfile)")
    print(s.getvalue())


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
