#!/usr/bin/env python3
"""Headline benchmark: the GA evaluation loop at population 65 536 per GPU.

--config wide runs BASELINE config 5 instead: the same generation step for the
wide MLP [6,512,512,3] (f32 genome storage, k_wide streaming kernel).

Secondary runs:
  --horizon T        the fixed-horizon measurement mode: every game slot runs
                     exactly T frames with auto-reset, nothing advanced in
                     closed form (pg_eval_args.horizon) -- the steady-state
                     env-steps/s (main.py:76-107's frames, every one stepped);
  --schedule reference  evaluate()'s own 6-game schedule (main.py:33-53: games
                     0-2 scripted / the 1-player CPU, games 3-5 vs the hall of fame);
  --dist init        U[0,1) genes (toolbox.attr_float = random.random, ga.py:85)
                     instead of the "evolved" N(0, 3).

One step = one GA generation of the reference's eaSimple loop
(main.py:165-170) on device:
  1. evaluate every genome's 6 self-play games to termination
     (pg_eval_population: Pong physics + both paddles' [6,64,3] MLPs, fused),
  2. all-gather the fitness over ranks (RCCL; N > 1 only),
  3. HallOfFame.update (DEAP semantics: pg_row_hash on device, pg_hof_update on the host),
  4. selTournament(tournsize = pop//4) + varAnd(cxBlend, mutGaussian) on device
(pong_amd.evolve.DeviceGA, the product's device-resident eaSimple).
Weak scaling: every rank evaluates 65 536 genomes of an N x 65 536 population.

Launch: python bench.py [--gpus N --steps K --warmup W]; N > 1 through
torch.distributed.run (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* from the env).
Rank 0 prints ONE JSON line.  Data: synthetic N(0, 3) genomes (the
"evolved" distribution of SURVEY 8d), seeded per rank layout.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "neuro-genetic-pong-self-play_amd")
sys.path.insert(0, PKG)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

F32_VECTOR_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: peak FP32 vector (= f32 MFMA) rate
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E peak
PROFILE_ROUND = "r06"           # profiles/<round>/ holds the PMC passes of the committed build


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="selfplay", choices=["selfplay", "wide"],
                   help="selfplay = BASELINE config 3 ([6,64,3], the headline); wide = config 5 ([6,512,512,3])")
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=None)
    p.add_argument("--warmup", type=int, default=None)
    p.add_argument("--pop", type=int, default=65536, help="genomes per GPU (selfplay, weak scaling) / in total (wide, strong scaling)")
    p.add_argument("--shape", default=None)
    p.add_argument("--games", type=int, default=6)
    p.add_argument("--dtype", default=None, choices=["float64", "float32"])
    p.add_argument("--group-lanes", type=int, default=0)
    p.add_argument("--kernel", default="auto")
    p.add_argument("--sigma", type=float, default=3.0)
    p.add_argument("--dist", default="normal", choices=["normal", "init"],
                   help="genes N(0, sigma) ('evolved', the headline) or U[0,1) ('init', ga.py:85)")
    p.add_argument("--schedule", default="selfplay", choices=["selfplay", "reference"],
                   help="selfplay: all-NN games vs the hall of fame (headline); reference: main.py:33-53's schedule")
    p.add_argument("--horizon", type=int, default=0,
                   help="T > 0: fixed-horizon mode, every game slot runs exactly T frames with auto-reset")
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--cpu-baseline-seconds", type=float, default=10.0)
    p.add_argument("--cpu-threads", type=int, default=16,
                   help="CPU baseline pool: this box's CPU share per GPU (the pool's rule on a one-GPU box)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    a = p.parse_args()
    wide = a.config == "wide"
    # presets: a wide generation takes ~30 s at 65 536 genomes, so fewer steps
    a.steps = a.steps if a.steps is not None else (1 if wide else 5)
    # two warm-up steps: the initial evaluation and one full generation (first-call costs of select/vary)
    a.warmup = a.warmup if a.warmup is not None else (0 if wide else 2)
    a.shape = a.shape or ("6,512,512,3" if wide else "6,64,3")
    a.dtype = a.dtype or ("float32" if wide else "float64")
    return a


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cpu_pool = None
    if world == 1 and not args.no_cpu_baseline:
        # the CPU baseline's worker processes are forked now, before anything touches the GPU
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import numpy_loop
        cpu_pool = numpy_loop.make_pool(args.cpu_threads)
    # PG_DIST_BACKEND=gloo with more ranks than GPUs: a rehearsal of the N > 1
    # path on a one-GPU box (ranks share devices); the driver's runs use RCCL
    backend = os.environ.get("PG_DIST_BACKEND", "nccl")
    local_dev = local % max(torch.cuda.device_count(), 1) if backend == "gloo" else local
    # PG_FORCE_DIST=1 runs the N > 1 path (process group, barriers, max-over-ranks
    # timing, the fitness all-gather) at any world size, e.g. RCCL at N = 1
    dist_on = world > 1 or os.environ.get("PG_FORCE_DIST") == "1"
    if dist_on:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local_dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_dev))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local_dev if dist_on else 0)
    torch.cuda.set_device(dev)

    from pong_amd import build as B
    from pong_amd import device as D
    from pong_amd.evolve import DeviceGA
    B.build()

    shape = [int(v) for v in args.shape.split(",")]
    dtype = torch.float64 if args.dtype == "float64" else torch.float32
    if args.config == "wide":
        # BASELINE config 5 is population 65 536 scaled over 1 -> 8 GPUs: strong
        # scaling (the replicated f32 state of 65 536 + 16 384 wide genomes is
        # ~175 GB per GPU, so the population cannot grow with N)
        P = args.pop
        n_local = -(-P // world)
    else:
        n_local = args.pop  # weak scaling: 65 536 genomes per GPU
        P = n_local * world
    H = max(P // 4, 1)                 # HALL_OF_FAME_AMOUNT = POPULATION_SIZE // 4 (config.py:49-50)
    tournsize = max(P // 4, 1)          # TOURNAMENT_SIZE (config.py:49)
    # the device-resident eaSimple (pong_amd.evolve): replicated population,
    # rank r evaluates its shard, one all-gather of fitness per generation;
    # GA parameters are config.py's (cxpb = mutpb = indpb = alpha = sigma = 0.9, mu = 0)
    # self-play: each GPU's block of n_local genomes plays its interleaved 1/N slice
    # of the hall (pg_schedule_args.hof_slices) -- the per-GPU work,
    # opponents included, stays that of N = 1 (K = 1 there: the plain schedule)
    ga = DeviceGA(shape, P, H, tournsize, dtype=dtype, device=dev, n_games=args.games, schedule=args.schedule,
                  seed=args.seed, kernel=args.kernel,
                  hof_block_rows=n_local if (args.config == "selfplay" and args.schedule == "selfplay") else 0)
    ga.ev.group_lanes = args.group_lanes
    ga.ev.horizon = args.horizon  # pg_eval_args.horizon: 0 = evaluate()'s episodes
    ga.order_by_length = os.environ.get("PG_NO_LENGTH_ORDER") != "1"  # A/B switch for the evaluation order
    ga.early_prep = os.environ.get("PG_NO_EARLY_PREP") != "1"  # A/B switch: schedule + genome records during the HoF scan
    ga.prepare_first = os.environ.get("PG_NO_PREPARE_FIRST") != "1"  # A/B switch: the HoF prepare before the side stream's work
    ga.presubmit = os.environ.get("PG_NO_PRESUBMIT") != "1"  # A/B switch: the next generation's side work enqueued before the merge sync
    ga.persistent_bufs = os.environ.get("PG_NO_PERSIST") != "1"  # A/B switch: schedule/invalid/remap buffers kept
    # config 5 (strong scaling): contiguous shards.  Length-balanced shards
    # (DeviceGA.balance_shards, PG_BALANCE=1) measured no better at P = 65 536:
    # 8 192 genomes a rank already even out (straggler factor 1.0016 contiguous
    # vs 1.0069 balanced at N = 8; profiles/r06/scale_model_wide.log)
    ga.balance_shards = args.config == "wide" and os.environ.get("PG_BALANCE") == "1"
    G = ga.G
    ga.initialize("normal" if args.dist == "normal" else "uniform", args.sigma)
    # the first games already face a full hall of fame: H independent random
    # genomes at fitness -1e300, which the first update replaces
    gen = torch.Generator(device=dev).manual_seed(args.seed + 1)
    rows = max(1, (1 << 28) // (8 * G))
    for r0 in range(0, H, rows):
        r1 = min(H, r0 + rows)
        if args.dist == "normal":
            blk = torch.randn((r1 - r0, G), generator=gen, dtype=torch.float64, device=dev).mul_(args.sigma)
        else:
            blk = torch.rand((r1 - r0, G), generator=gen, dtype=torch.float64, device=dev)
        ga.store[r0:r1] = blk.to(dtype)
    ga.set_hall_of_fame(None, np.full(H, -1e300))
    lo = ga.lo

    for w in range(args.warmup):
        ga.step()
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    steps_local = 0
    fwd_local = 0
    slow_local = 0
    cert_local = [0, 0, 0]  # certificate failures, decided by the f64 certificate, decided by the f32 plateau rule
    passes_local = 0        # k_wide: network weight passes (each streams one network's genes once)
    skip_local = 0          # episode frames of periodic rallies advanced at once (counters[8])
    hidden_local = 0        # serve-delay frames advanced at once (counters[12])
    counters = []
    events = []
    probe_local = [0, 0, 0]  # diagnostic builds (PG_DECIDE_PROBE, PG_START_PROBE): counters[13..15]
    for s in range(args.steps):
        # a fresh pair per step, read after the timed region: no per-step sync
        ga.eval_events = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        events.append(ga.eval_events)
        ga.step()  # evaluate + all-gather + hall of fame + select + vary (one generation)
        counters.append(ga.last.counters.clone())
    ga.eval_events = None
    torch.cuda.synchronize(dev)
    kernel_ms = [a.elapsed_time(b) for a, b in events]
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    for c in counters:
        c = c.cpu()
        steps_local += int(c[0])
        fwd_local += int(c[1])
        slow_local += int(c[2])
        for i in range(3):
            cert_local[i] += int(c[4 + i])
        passes_local += int(c[7])
        skip_local += int(c[8])
        hidden_local += int(c[12])
        probe_local = [a + int(v) for a, v in zip(probe_local, c[13:16])]

    t = torch.tensor([elapsed, float(steps_local), float(fwd_local), float(slow_local), sum(kernel_ms)]
                     + [float(v) for v in cert_local] + [float(passes_local), float(skip_local),
                                                          float(hidden_local)],
                     dtype=torch.float64, device=dev)
    if dist_on:
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        tsum = t.clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        elapsed = float(tmax[0])
        steps_all, fwd_all, slow_all = float(tsum[1]), float(tsum[2]), float(tsum[3])
        kernel_ms_mean = float(tsum[4]) / world / args.steps
        cert_all = [float(v) for v in tsum[5:8]]
        passes_all = float(tsum[8])
        skip_all = float(tsum[9])
        hidden_all = float(tsum[10])
    else:
        steps_all, fwd_all, slow_all = float(t[1]), float(t[2]), float(t[3])
        kernel_ms_mean = float(t[4]) / args.steps
        cert_all = [float(v) for v in t[5:8]]
        passes_all = float(t[8])
        skip_all = float(t[9])
        hidden_all = float(t[10])

    if rank == 0 and args.config == "wide":
        out = wide_report(args, world, shape, G, dtype, P, n_local, H, tournsize, elapsed, steps_all, fwd_all,
                          passes_all, kernel_ms_mean, skip_all)
        if not args.no_cpu_baseline and world == 1:  # the CPU baseline: rank 0 at N=1 only
            out["cpu_baseline"] = cpu_baseline(args, shape, ga, chunk=8, max_rows=256, pool=cpu_pool)
            cpu_pool.close()
        print(json.dumps(out), flush=True)
    elif rank == 0:
        # value = env-steps STEPPED frame by frame (physics + obs + every NN
        # forward of the frame) per second of wall time -- the
        # definition of BENCH_r02.  The episode frames the reference's
        # perform_episode loop runs (main.py:76-107) also count frames advanced
        # in closed form with bit-identical outcomes (periodic rallies to their
        # timeout, serve delays; tests/test_gpu_parity.py): a side field.
        # --horizon T steps every frame of every game slot (no closed form).
        stepped_all = steps_all
        episode_all = stepped_all + skip_all + hidden_all
        env_steps_per_s = stepped_all / elapsed
        ms_per_step = elapsed * 1000.0 / args.steps
        # roofline of the dominant kernel (k_service), per launch on rank 0's timing
        flops_per_forward = 2.0 * G
        fwd_per_launch = fwd_all / world / args.steps
        steps_per_launch = stepped_all / world / args.steps
        achieved_tflops = fwd_per_launch * flops_per_forward / (kernel_ms_mean / 1e3) / 1e12
        streaming_bytes = steps_per_launch * (2 * 4 * G + 128)   # SURVEY 8d accounting, GB-equivalent
        sched = ("self-play games vs the hall of fame" if args.schedule == "selfplay" else
                 "evaluate()'s schedule (main.py:33-53: HardcodedAi, the 1-player CPU, ScoreHardcodedAi, 3 hall-of-fame games)")
        mode = (f"fixed horizon: every game slot {args.horizon} frames, auto-reset (SURVEY 8d)" if args.horizon
                else "every game to termination (evaluate())")
        out = {
            "metric": "env-steps/sec (GA evaluation loop, self-play) + generations/sec at pop=65536 per GPU",
            "value": env_steps_per_s,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "generations_per_sec": 1000.0 / ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32 hidden + certified f64 argmax; genomes " + ("f64" if dtype == torch.float64 else "f32"),
            "data": "synthetic %s genomes, random-init [%s] MLPs, %s" % (
                "N(0,%g)" % args.sigma if args.dist == "normal" else "U[0,1) (ga.py:85 init)", args.shape, sched),
            "config": {"workload": "BASELINE config 3: population 65536 per GPU, MLP [6,64,3], 6 games per genome "
                                   "(%s), device GA step (selTournament/varAnd/HoF); %s" % (sched, mode),
                       "population": P, "population_per_gpu": n_local, "network_shape": shape,
                       "games_per_genome": args.games, "tournsize": tournsize, "hall_of_fame": H,
                       "schedule": args.schedule, "genes": args.dist, "horizon": args.horizon,
                       "parallelism": f"dp{world}" if world > 1 else "dp1",
                       "process_group": (dist.get_backend() if dist.is_initialized() else None),
                       "env_steps_definition": "env-steps stepped one frame at a time (physics, observation and "
                                               "every network forward of the frame); value = their count / wall "
                                               "time (BENCH_r02's definition)",
                       "env_steps_per_generation": stepped_all / args.steps,
                       "episode_env_steps_per_sec": episode_all / elapsed,
                       "episode_env_steps_per_generation": episode_all / args.steps,
                       "periodic_rally_frames_advanced_per_generation": skip_all / args.steps,
                       "serve_delay_frames_advanced_per_generation": hidden_all / args.steps,
                       "certificate_failures_per_forward": cert_all[0] / max(fwd_all, 1.0),
                       "failures_decided_in_wave": cert_all[2] / max(cert_all[0], 1.0),
                       "failures_decided_by_f64_certificate": cert_all[1] / max(cert_all[0], 1.0),
                       "numpy_order_f64_forwards_per_forward": slow_all / max(fwd_all, 1.0),
                       **({"probe_counters_13_15": probe_local} if probe_local[2] else {})},
            "roofline": _selfplay_roofline(args, G, dtype, achieved_tflops, kernel_ms_mean, flops_per_forward,
                                           fwd_per_launch, steps_per_launch, streaming_bytes, n_local, H),
        }
        if not args.no_cpu_baseline and world == 1:  # the CPU baseline: rank 0 at N=1 only
            out["cpu_baseline"] = cpu_baseline(args, shape, ga, pool=cpu_pool)
            cpu_pool.close()
        print(json.dumps(out), flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()


def _selfplay_roofline(args, G, dtype, achieved_tflops, kernel_ms_mean, flops_per_forward, fwd_per_launch,
                       steps_per_launch, streaming_bytes, n_local, H):
    """Roofline of k_service: compute-bound on the f32 vector ALU (VALU issue);
    HBM traffic from the committed PMC passes of the same build and command."""
    wt = 8 if dtype == torch.float64 else 4
    pmc, src = _pmc(_pmc_name(args))
    # MI355X_MICROARCH.md (HBM / rocprofv3): on gfx950 FETCH_SIZE counts half the
    # bytes of 16-B-per-lane reads -- the width of every k_service global load
    # (load_rec's float4 pieces of the lane records) -- so traffic = 2 x FETCH_SIZE
    # + WRITE_SIZE; the uncorrected sum is reported beside it
    traffic = pmc.get("traffic_bytes_fetch_x2") if pmc else None
    traffic_raw = pmc.get("traffic_bytes") if pmc else None
    stale = _pmc_stale(pmc)
    if stale:  # counters of another build: not this kernel's traffic
        traffic = traffic_raw = None
    unique = (n_local + H) * G * wt  # every genome row and hall-of-fame row once
    kernel_s = kernel_ms_mean / 1e3
    return {"bound": "valu", "achieved": achieved_tflops, "peak": F32_VECTOR_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": achieved_tflops / F32_VECTOR_PEAK_TFLOPS,
            "traffic": traffic,
            "hbm_GBps": traffic / kernel_s / 1e9 if traffic else None,
            "hbm_frac_of_peak": traffic / kernel_s / 1e9 / HBM_PEAK_GBS if traffic else None,
            "unique_row_bytes_per_launch": unique,
            "refetch_ratio": traffic / unique if traffic else None,
            "traffic_stale": stale,
            "traffic_uncorrected": traffic_raw,
            "traffic_note": "HBM-side bytes per launch (L2 memory-side requests, MALL hits included): rocprofv3 "
                            "2 x FETCH_SIZE + WRITE_SIZE of the same bench command, separate --pmc passes (%s); "
                            "FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950 rule for 16-B-per-lane reads "
                            "(traffic_uncorrected = FETCH_SIZE + WRITE_SIZE); each game loads both networks' lane "
                            "records, so genome rows are fetched ~refetch_ratio times; hbm_GBps = traffic / this "
                            "run's kernel time" % src,
            "engine": "compute-bound on the f32 vector ALU (v_pk_fma_f32, v_exp_f32, v_rcp_f32), no MFMA: every "
                      "game has its own 64x7 and 3x64 matrices applied to one input column; peak = MI355X f32 dense "
                      "peak (157.3 TF, equal for VALU and MFMA); the kernel is VALU-issue-bound: most VALU "
                      "instructions per env-step are physics, features, certificate and bookkeeping, not the "
                      "network's FMAs (DESIGN.md 4.1; SQ counters: profiles/%s/sq_summary_final.txt)" % PROFILE_ROUND,
            "kernel": "k_service<8,16,3,double> (pg_eval_population: 8 games per wave, 4 lanes per network, "
                      "8 game waves per block; certificate failures decided by the wave itself)",
            "kernel_ms_per_launch": kernel_ms_mean,
            "flops_per_forward": flops_per_forward,
            "forwards_per_launch": fwd_per_launch,
            "streaming_equivalent_GBps": streaming_bytes / kernel_s / 1e9,
            "streaming_equivalent_frac_of_hbm": streaming_bytes / kernel_s / 1e9 / HBM_PEAK_GBS}


def _pmc_name(args):
    """The PMC summary of this run's workload: the headline's, or a secondary run's."""
    tags = ([f"horizon{args.horizon}"] if args.horizon else []) + (["reference"] if args.schedule == "reference" else []) \
        + (["init"] if args.dist == "init" else [])
    return "pmc_traffic.json" if not tags else "pmc_traffic_%s.json" % "_".join(tags)


def wide_report(args, world, shape, G, dtype, P, n_local, H, tournsize, elapsed, steps_all, fwd_all, passes_all,
                kernel_ms_mean, skip_all=0.0):
    """BASELINE config 5: the generation step with the wide MLP; k_wide is
    HBM-bound (its W2 stream), so the roofline is bytes of weights streamed
    per launch over the launch time against the 8 TB/s HBM peak."""
    wt = 4 if dtype == torch.float32 else 8
    ms_per_step = elapsed * 1000.0 / args.steps
    passes_per_launch = passes_all / world / args.steps
    steps_per_launch = steps_all / world / args.steps
    bytes_per_launch = passes_per_launch * G * wt
    achieved = bytes_per_launch / (kernel_ms_mean / 1e3) / 1e9
    survey_bytes = steps_per_launch * (2 * 4 * G + 128)  # both networks streamed per env-step
    pmc, pmc_src = _pmc("pmc_traffic_wide.json")
    traffic = pmc.get("traffic_bytes_fetch_x2") if pmc else None
    stale = _pmc_stale(pmc)
    if stale:
        traffic = None
    return {
        "metric": "env-steps/sec (GA evaluation loop, self-play, wide MLP) + generations/sec at pop=65536",
        "value": steps_all / elapsed,  # env-steps stepped frame by frame (periodic rallies jumped: a side field)
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "generations_per_sec": 1000.0 / ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64 (numpy_nn's operation order); genomes " + ("f32" if wt == 4 else "f64"),
        "data": "synthetic N(0,%g) genomes, random-init [%s] MLPs, self-play vs hall of fame" % (args.sigma, args.shape),
        "config": {"workload": "BASELINE config 5: population 65536 in total (strong scaling over the GPUs), wide MLP [6,512,512,3], 6 self-play "
                               "games per genome, device GA step (selTournament/varAnd/HoF)",
                   "population": P, "population_per_gpu": n_local, "network_shape": shape,
                   "games_per_genome": args.games, "tournsize": tournsize, "hall_of_fame": H,
                   "parallelism": f"dp{world}" if world > 1 else "dp1",
                   "process_group": (dist.get_backend() if dist.is_initialized() else None),
                   "env_steps_definition": "env-steps stepped one frame at a time (physics, observation and "
                                           "every network forward of the frame); value = their count / wall time",
                   "env_steps_per_generation": steps_all / args.steps,
                   "episode_env_steps_per_sec": (steps_all + skip_all) / elapsed,
                   "episode_env_steps_per_generation": (steps_all + skip_all) / args.steps,
                   "periodic_rally_frames_advanced_per_generation": skip_all / args.steps,
                   "network_passes_per_generation": passes_all / args.steps,
                   "forwards_per_network_pass": fwd_all / max(passes_all, 1.0)},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_stale": stale,
                     "traffic_over_algorithmic": (traffic / bytes_per_launch) if traffic else None,
                     "traffic_note": "HBM bytes per launch from the PMC passes (%s): 2 x FETCH_SIZE + WRITE_SIZE "
                                     "(MI355X_MICROARCH.md: on gfx950 FETCH_SIZE counts half the bytes of 16-B-per-lane "
                                     "streaming loads, which the W2 stream is); includes the per-genome tile-major "
                                     "re-lay (one read + one write of each network's W2)" % (pmc_src or "none"),
                     "kernel": "k_wide<6,float> (pg_eval_population: one 512-thread workgroup per genome, six games "
                               "in lockstep; each network's W2 re-laid tile-major into the block's scratch at "
                               "genome start, then streamed HBM->registers once per frame per network with "
                               "line-aligned 1-KB non-temporal wave loads, no LDS staging)",
                     "kernel_ms_per_launch": kernel_ms_mean,
                     "bytes_per_network_pass": G * wt,
                     "network_passes_per_launch": passes_per_launch,
                     "survey_algorithmic_GBps": survey_bytes / (kernel_ms_mean / 1e3) / 1e9,
                     "note": "achieved = genome bytes streamed (network passes x genes x 4 B) / launch time; "
                             "survey_algorithmic counts both networks' genes per env-step (SURVEY 8d), which the "
                             "lockstep genome pass amortises over the genome's games",
                     **_measured_ceiling(achieved)},
    }


def _measured_ceiling(achieved_gbps):
    """The box's measured streaming-read ceiling beside the spec: the best rate
    of tools/hbm_ceiling.hip (k_wide's load shape -- 1-KB line-aligned
    non-temporal wave pieces, 512-thread blocks -- over an 8-16 GiB buffer read
    once per pass, far past the 256 MiB Infinity Cache) in
    profiles/<round>/hbm_ceiling.jsonl, when that run is on file."""
    path = os.path.join(REPO, "profiles", PROFILE_ROUND, "hbm_ceiling.jsonl")
    try:
        runs = [json.loads(line) for line in open(path) if line.strip()]
    except OSError:
        return {"measured_ceiling_GBps": None}
    best = max(runs, key=lambda r: r["best_TBps"])
    ceil = best["best_TBps"] * 1e3
    return {"measured_ceiling_GBps": ceil, "frac_of_measured_ceiling": achieved_gbps / ceil,
            "measured_ceiling_source": "profiles/%s/hbm_ceiling.jsonl: best of %d configurations (%d blocks of 512, "
                                       "%d pieces in flight per wave, %.0f GiB)"
                                       % (PROFILE_ROUND, len(runs), best["grid"], best["pieces_in_flight_per_wave"],
                                          best["bytes"] / 2**30)}


def cpu_baseline(args, shape, ga, chunk=256, max_rows=1 << 16, pool=None):
    """The reference's CPU path on the host cores: oracle/numpy_loop.py, the
    reference's per-frame numpy loop restated (main.py:69-112, utils.find_stuff,
    numpy_nn.NeuralNetwork.run; calibrated against the real reference in the
    build container: profiles/r02/cpu_calibration.json), on the same workload's
    first genomes and schedule, in a process pool and on one core.  The C
    restatement (oracle/pong_oracle.c, OpenMP) is reported beside it as
    ``c_port``."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    import numpy_loop as NL
    from pong_amd import device as D
    O.build()
    lo = ga.lo
    # host copies bounded by bytes (a wide genome is 2.1 MB in f64): at most
    # 1 GiB of genomes, per pool worker at most 16 MiB of them (and only the
    # opponent rows its own games use), C-port chunks of at most 64 MiB
    row_bytes = ga.G * 8
    max_rows = max(8, min(max_rows, (1 << 30) // row_bytes))
    per_worker = max(2, min(64, (16 << 20) // row_bytes))
    chunk = max(1, min(chunk, (64 << 20) // row_bytes))
    genomes = ga.shard_rows()[:max_rows].double().cpu().numpy()
    n = genomes.shape[0]
    kind, opp, mult = D.schedule(ga.schedule, n, ga.n_games, lo, ga.hof_fitness, ga.hof_n, ga.seed,
                                 ga.generation + 1, ga.device)
    hof = ga.hall_of_fame
    k, o, m = kind.cpu().numpy(), opp.cpu().numpy(), mult.cpu().numpy()
    # only the hall-of-fame rows these genomes play (the wide HoF is 35 GB in f64)
    rows = np.unique(o)
    opponents = hof[torch.as_tensor(rows, device=hof.device)].double().cpu().numpy()
    o = np.searchsorted(rows, o).astype(np.int32)
    secs = args.cpu_baseline_seconds
    workers = args.cpu_threads
    # numpy loop on `workers` processes, then on one core (~secs and ~secs/2 of wall time)
    np_rows = min(n, per_worker * workers)
    # the one-core leg: worker 0's own games replayed alone in one pool process
    # afterwards (the same sample from its start, nothing else running)
    rate_p, steps_p, games_p, dt_p, solo = NL.timed_rate(shape, genomes[:np_rows], k[:np_rows], o[:np_rows],
                                                         m[:np_rows], opponents, secs, workers, pool,
                                                         solo_seconds=secs / 2)
    rate_1, steps_1, games_1, dt_1, w0_pooled = solo
    # the C restatement with OpenMP
    steps, done = 0, 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < secs / 2 and done + chunk <= genomes.shape[0]:
        r = O.eval_population(genomes[done:done + chunk], shape, k[done:done + chunk], o[done:done + chunk],
                              m[done:done + chunk], opponents=opponents, n_threads=workers)
        steps += int(r["frames"].sum())
        done += chunk
    dt = time.perf_counter() - t0
    return {"value": rate_p, "unit": "env-steps/s", "cores": workers, "kind": "port",
            "sample": f"the reference's per-frame numpy loop (oracle/numpy_loop.py) on {workers} worker processes, "
                      f"one BLAS thread each: {games_p} whole games of the same workload's first genomes "
                      f"({steps_p} env-steps; each worker timed on its own clock, at most {dt_p:.1f} s; value = "
                      f"the sum of the workers' rates); {workers} = this box's CPU share per GPU",
            "one_core": {"value": rate_1, "sample": f"worker 0's games of the pooled run, replayed alone in one "
                                                     f"process: {games_1} games, {steps_1} env-steps in {dt_1:.1f} s",
                         "worker0_in_pool": w0_pooled},
            "calibration": "numpy_loop runs 1.11x the reference's own rate on the same games, equal rewards "
                           "(profiles/r02/cpu_calibration.json)",
            "c_port": {"value": steps / dt if dt > 0 else None, "cores": workers,
                       "sample": f"C restatement (oracle/pong_oracle.c, OpenMP over {workers} threads): "
                                 f"{done} genomes x {args.games} games ({steps} env-steps in {dt:.1f} s)"},
            "cpu": _cpu_model(),
            "host_cpus": _host_cpus(workers),
            "full_box": _full_box(rate_p, workers)}


def _full_box(rate_p, workers):
    """SURVEY 8(d)'s whole-node CPU figure: os.cpu_count() cores at the pooled
    per-core rate.  Extrapolated, not run -- the job's cgroup grants 16 CPUs of
    time (``host_cpus``), and a pool of os.cpu_count() processes would
    time-slice those same 16."""
    n = os.cpu_count() or workers
    per_core = rate_p / workers if workers else None
    return {"cores": n, "value": per_core * n if per_core else None, "per_core": per_core,
            "kind": "extrapolated: pooled per-core rate x os.cpu_count()"}


def _pmc(name):
    """The newest committed PMC summary of this name (profiles/<round>/), and its path."""
    for rnd in (PROFILE_ROUND,):
        path = os.path.join("profiles", rnd, name)
        try:
            with open(os.path.join(REPO, path)) as fh:
                return json.load(fh), path
        except (OSError, ValueError):
            continue
    return None, None


def _lib_sha():
    import hashlib
    from pong_amd import _lib as L
    with open(L.LIB_PATH, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]


def _pmc_stale(pmc):
    """None when the committed PMC summary was taken on the library this run
    loaded; else why not (bench then reports no traffic)."""
    if not pmc:
        return "no PMC summary"
    want = pmc.get("lib_sha256_16")
    if not want:
        return "PMC summary names no library build"
    have = _lib_sha()
    return None if want == have else f"PMC summary of build {want}, this run loaded {have}"


def _pmc_traffic(name="pmc_traffic.json"):
    pmc, _ = _pmc(name)
    return pmc.get("traffic_bytes") if pmc else None


def _host_cpus(workers):
    """What the box lets this job use (SURVEY 8(d) asks for a pool of
    os.cpu_count() processes): the visible CPUs, this process's affinity, and
    the cgroup's CPU quota -- on the MI355X boxes os.cpu_count() shows the whole
    node (256) while cpu.max grants 16 CPUs of time, so a 16-process pool is the
    full box available to the job and a larger pool would only time-slice it."""
    out = {"os_cpu_count": os.cpu_count(), "pool_processes": workers}
    try:
        out["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
        out["cgroup_cpu_max"] = f"{q} {per}"
        if q != "max":
            out["cgroup_cpus"] = int(q) / int(per)
    except (OSError, ValueError):
        pass
    quota = out.get("cgroup_cpus")
    out["pool_is_full_quota"] = bool(quota is not None and workers >= quota)
    return out


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main()
