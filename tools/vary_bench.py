#!/usr/bin/env python3
"""Time k_vary (pg_ga_vary, varAnd) alone: P offspring rows of [6,64,3] f64
genomes from random parents, HIP events over 20 launches.
usage: [PONG_GA_LIB=...] python tools/vary_bench.py [P ...]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "neuro-genetic-pong-self-play_amd"))

import torch  # noqa: E402

from pong_amd import device as D  # noqa: E402


def main(argv):
    dev = torch.device("cuda", 0)
    G = 454
    for P in [int(v) for v in argv] or [65536, 524288]:
        parents = torch.randn((P, G), dtype=torch.float64, device=dev) * 3
        out = torch.empty_like(parents)
        chosen = torch.randint(0, P, (P,), dtype=torch.int32, device=dev)
        args = (parents, chosen, G, 0.5, 0.2, 0.5, 0.0, 1.0, 0.1)
        for w in range(3):
            D.vary(*args, seed=1, generation=w, out=out)
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for r in range(20):
            D.vary(*args, seed=1, generation=10, out=out)
        t1.record()
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / 20
        print(json.dumps({"lib": os.path.basename(os.environ.get("PONG_GA_LIB", "default")), "P": P, "ms": ms,
                          "GBps": 2 * P * G * 8 / (ms * 1e6),
                          "checksum": float(out.sum())}), flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
