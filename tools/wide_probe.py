#!/usr/bin/env python3
"""Time k_wide on a [6,512,512,3] self-play population (one launch) and print
env-steps/s, network passes and the weight bytes they streamed.
usage: python tools/wide_probe.py [pop] [hof] [dtype]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "neuro-genetic-pong-self-play_amd"))

import torch  # noqa: E402

from pong_amd import device as D  # noqa: E402

pop = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
hof = int(sys.argv[2]) if len(sys.argv) > 2 else max(pop // 4, 1)
dtype = torch.float32 if (len(sys.argv) <= 3 or sys.argv[3] == "f32") else torch.float64
shape = [int(v) for v in os.environ.get("PG_SHAPE", "6,512,512,3").split(",")]
dev = torch.device("cuda", 0)
ev = D.Evaluator(shape, dtype=dtype, device=dev, kernel=os.environ.get("PG_KERNEL", "wide"))
gen = torch.Generator(device=dev).manual_seed(1234)
genomes = (torch.randn((pop, ev.genes), generator=gen, dtype=torch.float64, device=dev) * 3.0).to(dtype)
opponents = genomes[:hof].contiguous()
kind, opp, mult = ev.selfplay_schedule(pop, hof)
for rep in range(2):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    res, _ = ev.evaluate(genomes, kind, opp, mult, opponents=opponents, validate=False)
    e1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ms = e0.elapsed_time(e1)
    c = res.counters.cpu().tolist()
    wb = c[7] * ev.genes * genomes.element_size()
    print(f"rep {rep}: pop {pop} hof {hof} {ms:.1f} ms (wall {wall*1e3:.1f}), env-steps {c[0]} "
          f"({c[0] / (ms / 1e3):.3e}/s), forwards {c[1]}, games {c[3]}, network passes {c[7]}, "
          f"weight bytes {wb:.3e} = {wb / (ms / 1e3) / 1e9:.0f} GB/s, "
          f"frames/game mean {res.frames.float().mean().item():.0f} max {res.frames.max().item()}", flush=True)
    if any(c[4:7]):  # diagnostic build: shader-clock cycles per phase, summed over workgroups
        tot = sum(c[4:7])
        print("   phase cycles share: A+E+B %.3f  C %.3f  D %.3f" % tuple(v / tot for v in c[4:7]), flush=True)
