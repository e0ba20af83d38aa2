#!/usr/bin/env python3
"""Phase timing of k_staged on the bench workload (diagnostic).

Needs a library built with -DPG_STAGED_PROFILE (PG_TU=pg_staged.hip
tools/build_variant.sh prof -DPG_STAGED_PROFILE), picked with PONG_GA_LIB.
The kernel then writes per-block cycle counts into the trace buffer:
[0] frames, [1] env cycles waiting for the network stage (incl. service),
[2] service cycles, [3] env cycles wait + phase C + phase A, [4] env barrier
cycles, [5] net wave 0 compute cycles, [6] net wave 0 barrier cycles,
[7] block cycles, [8] playing slot-frames, [9] visible slot-frames,
[10] requests served, [11] env cycles before the wait (overlapped start pipeline),
[16 + w] network wave w's compute cycles.
usage: PONG_GA_LIB=variants/lib_prof.so python tools/staged_probe.py
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "neuro-genetic-pong-self-play_amd"))


def main():
    from pong_amd.device import Evaluator
    dev = torch.device("cuda", 0)
    shape = [6, 64, 3]
    n, H = 65536, 16384
    ev = Evaluator(shape, device=dev, kernel="staged")
    gen = torch.Generator(device=dev).manual_seed(1234)
    genomes = torch.randn((n, ev.genes), generator=gen, dtype=torch.float64, device=dev) * 3.0
    hof = genomes[:H].contiguous()
    kind, opp, mult = ev.selfplay_schedule(n, H)
    nb = 256
    for rep in range(2):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        res, tr = ev.evaluate(genomes, kind, opp, mult, opponents=hof, trace_games=nb, trace_cap=256, validate=False)
        b.record()
        torch.cuda.synchronize()
    d = tr.cpu().numpy().view(np.uint64).reshape(nb, 32).astype(np.float64)
    fr = d[:, 0]
    out = {"kernel_ms": a.elapsed_time(b), "blocks": nb, "frames_per_block_mean": float(fr.mean()),
           "frames_per_block_max": float(fr.max()), "block_cycles_mean": float(d[:, 7].mean()),
           "cycles_per_frame": float((d[:, 7] / np.maximum(fr, 1)).mean())}
    names = {1: "env_wait", 2: "service", 3: "env_frame_to_barrier", 4: "env_barrier", 5: "net0_compute",
             6: "net0_barrier", 11: "env_pre_wait", 12: "done_detect_lag", 13: "net_stage_span"}
    for i, nm in names.items():
        out[nm + "_per_frame"] = float(d[:, i].sum() / fr.sum())
    out["env_C_A_per_frame"] = (out["env_frame_to_barrier_per_frame"] - out["env_wait_per_frame"]
                                - out["env_pre_wait_per_frame"])
    out["playing_slots_per_frame"] = float(d[:, 8].sum() / fr.sum())
    out["visible_slots_per_frame"] = float(d[:, 9].sum() / fr.sum())
    out["requests_per_frame"] = float(d[:, 10].sum() / fr.sum())
    out["net_wave_compute_per_frame"] = [float(d[:, 16 + w].sum() / fr.sum()) for w in range(7)]
    out["env_steps"] = int(res.counters[0])
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
