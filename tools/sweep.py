#!/usr/bin/env python3
"""Kernel-variant sweep for pg_eval_population on one GPU.

Runs each (library build, group_lanes) pair in its own process (the library
is picked with PONG_GA_LIB) on the bench workload -- pop 65 536, [6,64,3],
6 self-play games per genome vs a 16 384-row hall of fame -- and prints one
JSON line per variant: kernel ms per launch (HIP events), env-steps/s,
f64 re-decision rate.
usage: python tools/sweep.py --libs a.so,b.so --lanes 16,32,64 [--reps 3]
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(args):
    sys.path.insert(0, os.path.join(REPO, "neuro-genetic-pong-self-play_amd"))
    import torch
    from pong_amd.device import Evaluator
    dev = torch.device("cuda", 0)
    shape = [int(v) for v in args.shape.split(",")]
    n, H = args.pop, args.pop // 4
    ev = Evaluator(shape, device=dev, group_lanes=args.lane, kernel=args.kernel,
                   dtype=torch.float64 if args.dtype == "f64" else torch.float32)
    gen = torch.Generator(device=dev).manual_seed(1234)
    if args.dist == "uniform":  # toolbox.attr_float = random.random (ga.py:85): bench.py --dist init
        genomes = torch.rand((n, ev.genes), generator=gen, dtype=torch.float64, device=dev).to(ev.dtype)
    else:
        genomes = (torch.randn((n, ev.genes), generator=gen, dtype=torch.float64, device=dev) * args.sigma).to(ev.dtype)
    hof = genomes[:H].contiguous()
    kind, opp, mult = ev.selfplay_schedule(n, H)
    res, _ = ev.evaluate(genomes, kind, opp, mult, opponents=hof)
    torch.cuda.synchronize()
    ms, steps, slow, fwd = [], 0, 0, 0
    for _ in range(args.reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        res, _ = ev.evaluate(genomes, kind, opp, mult, opponents=hof, out=res, validate=False)
        b.record()
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b))
        c = res.counters.cpu()
        steps, fwd, slow, fails, plateau, tight = int(c[0]), int(c[1]), int(c[2]), int(c[4]), int(c[5]), int(c[6])
        passes = int(c[7])  # k_wide: network weight passes (each streams one network's genes once)
        c10, c11 = int(c[10]), int(c[11])  # k_wide stamps build: D and prep cycles
        rally, hidden = int(c[8]), int(c[12])
        probe = [int(c[13]), int(c[14]), int(c[15])]  # PG_START_PROBE build: start cycles, wave cycles, waves
    mean = sum(ms) / len(ms)
    print(json.dumps({"lib": os.path.basename(os.environ.get("PONG_GA_LIB", "default")), "lanes": args.lane,
                      "dist": args.dist,
                      "kernel": args.kernel,
                      "shape": shape, "kernel_ms": mean, "min_ms": min(ms), "env_steps": steps,
                      "env_steps_per_s": steps / (mean / 1e3), "fwd": fwd, "f64_redecide": slow,
                      "cert_fail": fails, "inwave_plateau": tight, "service_certified": plateau,
                      "memo_hits": fails - tight - plateau - slow, "passes": passes, "c10": c10, "c11": c11,
                      "rally_frames": rally, "hidden_frames": hidden, "start_probe": probe,
                      "episode_frames_per_s": (steps + rally + hidden) / (mean / 1e3),
                      "stream_TBps": passes * ev.genes * ev.dtype.itemsize / (mean / 1e3) / 1e12}), flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--libs", default="")
    p.add_argument("--lanes", default="16,32,64")
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--pop", type=int, default=65536)
    p.add_argument("--shape", default="6,64,3")
    p.add_argument("--sigma", type=float, default=3.0)
    p.add_argument("--dtype", default="f64")
    p.add_argument("--dist", default="normal", choices=("normal", "uniform"))
    p.add_argument("--kernel", default="split")
    p.add_argument("--one", action="store_true")
    p.add_argument("--lane", type=int, default=0)
    args = p.parse_args()
    if args.one:
        return one(args)
    libs = [l for l in args.libs.split(",") if l] or [""]
    for lib in libs:
        for lane in [int(v) for v in args.lanes.split(",")]:
            env = dict(os.environ)
            if lib:
                env["PONG_GA_LIB"] = os.path.abspath(lib)
            cmd = [sys.executable, __file__, "--one", f"--lane={lane}", "--reps", str(args.reps),
                   "--pop", str(args.pop), "--shape", args.shape, "--sigma", str(args.sigma), "--dtype", args.dtype,
                   "--kernel", args.kernel, "--dist", args.dist]
            r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
            if r.returncode != 0:
                print(json.dumps({"lib": lib, "lanes": lane, "error": r.stderr[-800:]}), flush=True)
                if r.returncode in (-6, -11, 134, 139):
                    sys.exit(r.returncode)
            else:
                print(r.stdout.strip(), flush=True)


if __name__ == "__main__":
    main()
