#!/usr/bin/env python3
"""Weak-scaling projection of bench.py to N GPUs, measured on one GPU.

BASELINE config 4 (P = N x 65 536 over N GPUs): every rank evaluates its
shard of 65 536 genomes and repeats the replicated eaSimple work of the whole
population (select/vary of P rows, the hall-of-fame update) -- DESIGN.md 7.
A rank varies only the offspring rows it needs (sharded variation,
evolve.DeviceGA.shard_vary).  This tool measures both terms on one GPU at
P = N x 65 536:
  * per-shard evaluation: after each DeviceGA generation, the shard of every
    rank is evaluated ON ITS OWN (the same rows, schedule and hall of fame a
    rank would play; one launch each, HIP events): the slowest shard sets the
    generation's pace at N (the straggler term), the mean is what N = 1 pays;
  * replicated work: the one-GPU generation's wall time minus its
    evaluation (the fused step's own events) at 65 536, plus the critical
    path of a rank's non-evaluation ops at P = N x 65 536 (op by op, sharded
    variation) beyond the same ops at 65 536;
and prints the projected efficiency (N=1 generation time) / (N generation time)
with t_N = max-shard eval + replicated(P) + all-gather(P) and t_1 = the MEASURED
one-GPU generation at 65 536 (the bench's own step: median wall time, round-5
review), and the same in env-steps/s: (sum of the shards' stepped env-steps /
t_N) / (N x the one-GPU generation's stepped env-steps / t_1).  Every shard and
the one-GPU evaluation report their stepped env-steps and ps per env-step, so a
slower shard is split into more frames vs slower frames.  The all-gather (fitness f64 + lineage f32 per row)
is priced at 1 TB/s aggregate over xGMI (a conservative reading of 7 x 153
GB/s links) plus 30 us.

usage: python tools/scale_model.py [N=8] [generations=6]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "neuro-genetic-pong-self-play_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pong_amd import device as D  # noqa: E402
from pong_amd.evolve import DeviceGA  # noqa: E402


def make_ga(P, dev, seed=1234, sigma=3.0):
    # bench.py's schedule: each 65 536-row block plays its slice of the hall (K = P / 65 536)
    ga = DeviceGA([6, 64, 3], P, device=dev, schedule="selfplay", seed=seed, hof_block_rows=65536)
    ga.initialize("normal", sigma)
    gen = torch.Generator(device=dev).manual_seed(seed + 1)
    rows = max(1, (1 << 28) // (8 * ga.G))
    for r0 in range(0, ga.H, rows):
        r1 = min(ga.H, r0 + rows)
        ga.store[r0:r1] = torch.randn((r1 - r0, ga.G), generator=gen, dtype=torch.float64, device=dev).mul_(sigma)
    ga.set_hall_of_fame(None, np.full(ga.H, -1e300))
    return ga


def timed_steps(ga, steps):
    """(wall ms, evaluation ms, stepped env-steps) per generation, steady state."""
    out = []
    for _ in range(steps):
        ga.eval_events = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ga.step()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        out.append((wall, ga.eval_events[0].elapsed_time(ga.eval_events[1]), int(ga.last.counters[0].item())))
    ga.eval_events = None
    return out


def shard_evals(ga, n_shards):
    """Each rank's shard of the current population evaluated on its own:
    (ms, stepped env-steps, opponents' record prep ms) each."""
    P, S = ga.P, ga.P // n_shards
    ev = D.Evaluator(ga.nodes, dtype=ga.dtype, device=ga.device, n_games=ga.n_games, seed=ga.ev.seed)
    K = ga.hof_slices
    hof = ga.hall_of_fame  # (items order; the in-place hall's rows gathered once)
    ms = []
    for r in range(n_shards):
        lo = r * S
        # what rank r plays: its block's slice of the hall (bench.py's schedule)
        sliced = K > 1 and ga.hof_n >= K and S == ga.hof_block_rows
        opponents = hof[r % K::K] if sliced else hof[: ga.hof_n]
        kind, opp, mult = D.schedule("selfplay", S, ga.n_games, lo, ga.hof_fitness, ga.hof_n, ga.seed,
                                     ga.generation + 1, ga.device, hof_slices=K, block_rows=ga.hof_block_rows,
                                     slice_local=sliced)
        rows = ga._rows[lo:lo + S]
        ev.evaluate(rows, kind, opp, mult, opponents=opponents, validate=False)  # warm (workspace)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        res, _ = ev.evaluate(rows, kind, opp, mult, opponents=opponents, validate=False)
        b.record()
        torch.cuda.synchronize()
        t = a.elapsed_time(b)
        # the genome records alone (prep="genomes" plays nothing): the rest of the
        # launch's preparation is the opponents' records (the hall of fame, P/4 rows)
        c, d = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c.record()
        ev.evaluate(rows, kind, opp, mult, opponents=opponents, validate=False, prep="genomes")
        d.record()
        torch.cuda.synchronize()
        ms.append((t, int(res.counters[0].item()), c.elapsed_time(d)))
    return ms


def replicated_ops(ga, n_shards=1, reps=3):
    """Device ms of a rank's generation work outside its evaluation, one op at
    a time on the GA's current state (HIP events, median of reps): merge of P
    fitness values, selTournament by rank sampling, varAnd (n_shards > 1:
    sharded variation -- shard 0's rows, then the completion: the candidates'
    and the next parents' pairs marked and varied, evolve.DeviceGA._complete),
    the clones' inherited fitness, the hall-of-fame candidates' prepare
    (hashes, ranks), the new members' commit; and the host scan."""
    P, dev = ga.P, ga.device
    out = {}

    def timed(name, fn):
        ms = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            r = fn()
            b.record()
            torch.cuda.synchronize()
            ms.append(a.elapsed_time(b))
        out[name] = float(np.median(ms))
        return r

    fit = ga.fitness.clone()
    worst = float(ga._hof_fit_host[-1]) if ga.hof_n >= ga.H else None
    new_fit = torch.empty_like(fit)
    cand = torch.empty(P, dtype=torch.int32, device=dev)
    cand_fit = torch.empty(P, dtype=torch.float64, device=dev)
    summ = torch.empty(8, dtype=torch.float64, device=dev)
    # fitness perturbed so that a steady-state share of rows beats the worst member
    timed("merge", lambda: D.merge_fitness(fit, None, None, new_fit, worst, cand, cand_fit, summ, ga.ws))
    k = int(summ[6].item())
    out["candidates"] = k
    chosen = torch.empty(P, dtype=torch.int32, device=dev)
    timed("select_ranked", lambda: D.select_ranked(fit, P, ga.tournsize, ga.seed, 99, ga.ws, chosen=chosen))
    offspring = ga.spare[ga.H:]
    kw = dict(seed=ga.seed, generation=99, out=offspring)
    args = (ga._rows, chosen, ga.G, ga.cxpb, ga.mutpb, ga.alpha, ga.mu, ga.sigma, ga.indpb)
    if n_shards == 1:
        timed("vary", lambda: D.vary(*args, **kw))
    else:
        pairs = (P + 1) // 2
        hi = P // n_shards
        skip = (0, (hi + 1) >> 1)
        shard = torch.zeros(pairs, dtype=torch.uint8, device=dev)
        shard[skip[0]:skip[1]] = 1
        timed("vary", lambda: D.vary(*args, **kw, pair_mask=shard))
        cmask = torch.empty(pairs, dtype=torch.uint8, device=dev)
        pmask = torch.empty(pairs, dtype=torch.uint8, device=dev)
        inv = torch.empty(P, dtype=torch.uint8, device=dev)

        lst = torch.empty(pairs, dtype=torch.int32, device=dev)
        cnt = torch.empty(1, dtype=torch.int32, device=dev)

        def complete(mask, rows, exclude=None):  # as evolve.DeviceGA._complete: mark, list, vary the list
            mask.zero_()
            D.mark_pairs(mask, rows, skip=skip, exclude=exclude)
            D.list_pairs(mask, lst, cnt)
            D.vary(*args, **kw, pair_list=(lst, cnt, min(rows.numel(), pairs)), invalid=inv)
        timed("complete_cand", lambda: complete(cmask, cand[:k]))
        timed("complete_parents", lambda: complete(pmask, chosen, cmask))
        out["complete_cand_pairs"] = int(cmask.sum().item())
        out["complete_parent_pairs"] = int(pmask.sum().item())
        out["distinct_parents"] = int(torch.unique(chosen).numel())
    inherited = torch.empty(P, dtype=torch.float64, device=dev)
    lin = torch.empty(P, dtype=torch.float32, device=dev)
    timed("inherit", lambda: D.inherit(chosen, fit, inherited, ga.lineage_frames, lin))
    if k:
        old_n = ga.hof_n
        ch = torch.empty(k, dtype=torch.int64, device=dev)
        pk = torch.empty(old_n + 2 * k, dtype=torch.int64, device=dev)
        timed("hof_prepare", lambda: D.hof_prepare_cand(ga.hof_fitness[:old_n], ga.hof_hash[:old_n], cand[:k],
                                                       cand_fit[:k], ga._rows, ga.G, ch, pk, ga.ws))
        pk_h = pk.cpu().numpy()
        n = old_n + k
        # the scan DeviceGA runs (pg_hof_update_packed straight on the device's
        # packing, with the in-place hall's slots), and beside it the general
        # scan it replaced (pg_hof_update)
        in_place = ga._in_place()
        t0 = time.perf_counter()
        r = D.hof_update_packed(ga.H, ga._hof_fit_host, pk_h, k, slot_in=ga._hof_slot_h if in_place else None,
                                slots=in_place)
        out["hof_scan_host"] = (time.perf_counter() - t0) * 1e3
        src, nf = r[0], r[1]
        t0 = time.perf_counter()
        D.hof_update(ga.H, ga._hof_fit_host, (pk_h[:old_n] >> 32), pk_h[n:].view(np.float64),
                     pk_h[old_n:n] >> 32, rank=(pk_h[:n] & 0xFFFFFFFF).astype(np.int32))
        out["hof_scan_host_general"] = (time.perf_counter() - t0) * 1e3
        m = src.shape[0]
        out["hof_entering"] = int((src >= old_n).sum())
        src_d = torch.tensor(src, dtype=torch.int32, device=dev)
        nf_d = torch.tensor(nf, dtype=torch.float64, device=dev)
        hh = torch.empty(max(m, 1), dtype=torch.int64, device=dev)
        hf = torch.empty(max(m, 1), dtype=torch.float64, device=dev)
        if in_place:  # into a copy of the hall: the GA's own state stays as it is
            hall = ga._hall_buf.clone()
            slot_d = torch.tensor(r[2], dtype=torch.int32, device=dev)
            timed("hof_commit", lambda: D.hof_commit(hall, None, ga._rows, cand[:k], src_d, old_n, ga.G,
                                                     ga.hof_hash, ch, hh, nf_d, hf, dst_slot=slot_d))
            del hall
        dst = torch.empty((m, ga.G), dtype=ga.dtype, device=dev)
        timed("hof_commit_dense" if in_place else "hof_commit",
              lambda: D.hof_commit(dst, ga.store, ga._rows, cand[:k], src_d, old_n, ga.G,
                                   ga.hof_hash, ch, hh, nf_d, hf))
        del dst
        if in_place and n_shards > 1:
            # a rank's slice of the in-place hall (its block plays hall[b::N]):
            # gathered in position order before its evaluation
            idx = ga.hof_slot[0:ga.hof_n:n_shards].long()
            sl = torch.empty((idx.shape[0], ga.G), dtype=ga.dtype, device=dev)
            timed("hall_slice_gather", lambda: torch.index_select(ga._hall_buf, 0, idx, out=sl))
            del sl
    # on the critical path: merge, the candidates' completion (sharded), their
    # prepare and commit; the selection, the parents' completion, the shard's
    # variation and inheritance run on the side stream beside the host scan
    # (evolve.py)
    dev_serial = (out.get("merge", 0) + out.get("complete_cand", 0) + out.get("hof_prepare", 0)
                  + out.get("hof_commit", 0) + out.get("hall_slice_gather", 0))
    side = out["select_ranked"] + out.get("complete_parents", 0) + out["vary"] + out["inherit"]
    overlapped = max(side, out.get("hof_scan_host", 0.0))
    out["replicated_critical_ms"] = dev_serial + overlapped
    # the code's stream structure (evolve._hof_update_fused): the side stream
    # starts right after the candidates' completion and runs beside the
    # prepare, the host scan and the commit; the slice gather follows both
    main = out.get("hof_prepare", 0) + out.get("hof_scan_host", 0) + out.get("hof_commit", 0)
    out["replicated_critical_ms_streams"] = (out.get("merge", 0) + out.get("complete_cand", 0)
                                             + out.get("hall_slice_gather", 0) + max(side, main))
    return out


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    gens = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    dev = torch.device("cuda", 0)
    S = 65536
    res = {"N": N, "shard": S}
    # replicated work at one GPU's population
    ga1 = make_ga(S, dev)
    for _ in range(3):
        ga1.step()
    t1 = timed_steps(ga1, gens)
    res["p65536_wall_ms"] = [w for w, _, _ in t1]
    res["p65536_eval_ms"] = [e for _, e, _ in t1]
    res["p65536_steps"] = [n for _, _, n in t1]
    res["p65536_ps_per_step"] = [e * 1e9 / n for _, e, n in t1]
    sh1 = shard_evals(ga1, 1)
    res["p65536_own_eval"] = {"ms": sh1[0][0], "steps": sh1[0][1], "genome_prep_ms": sh1[0][2],
                              "ps_per_step": sh1[0][0] * 1e9 / sh1[0][1]}
    print(json.dumps({"p65536": {k: res[k] for k in ("p65536_wall_ms", "p65536_eval_ms", "p65536_steps",
                                                     "p65536_ps_per_step", "p65536_own_eval")}}), flush=True)
    ops1 = replicated_ops(ga1, 1)
    print(json.dumps({"replicated_ops_p65536": ops1}), flush=True)
    res["replicated_ops_p65536"] = ops1
    del ga1
    torch.cuda.empty_cache()
    # the N-GPU population on one GPU
    gaN = make_ga(N * S, dev)
    for _ in range(3):
        gaN.step()
    walls, evals, shards = [], [], []
    for g in range(gens):
        (w, e, _), = timed_steps(gaN, 1)
        walls.append(w)
        evals.append(e)
        sh = shard_evals(gaN, N)
        shards.append(sh)
        print(json.dumps({"gen": gaN.generation, "wall_ms": w, "eval_ms": e, "shard_ms": [x[0] for x in sh],
                          "shard_steps": [x[1] for x in sh],
                          "shard_ps_per_step": [x[0] * 1e9 / x[1] for x in sh],
                          "shard_genome_prep_ms": [x[2] for x in sh]}), flush=True)
    ops = replicated_ops(gaN, N)
    print(json.dumps({"replicated_ops_pN": ops}), flush=True)
    res["replicated_ops_pN"] = ops
    # Why the one-GPU run at P has a longer non-evaluation wall than the model's
    # rank: it prepares the lane records of all P genomes (during the hall-of-
    # fame scan, outside the evaluation's events) where a rank prepares its
    # shard's, and its per-row order / scatter passes run over P rows.  The
    # P-row genome preparation, timed against a shard's:
    ev = D.Evaluator(gaN.nodes, dtype=gaN.dtype, device=dev, n_games=gaN.n_games, seed=gaN.ev.seed)
    kind, opp, mult = D.schedule("selfplay", gaN.P, gaN.n_games, 0, gaN.hof_fitness, gaN.hof_n, gaN.seed,
                                 gaN.generation + 1, dev)
    prep = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        ev.evaluate(gaN._rows, kind, opp, mult, opponents=gaN.hall_of_fame[:gaN.hof_n], validate=False,
                    prep="genomes")
        b.record()
        torch.cuda.synchronize()
        prep.append(a.elapsed_time(b))
    res["genome_prep_ms_all_P"] = float(np.median(prep))
    res["genome_prep_ms_shard"] = float(np.median([s[0][2] for s in shards]))
    del ev
    # the other per-row side-stream work of the one-GPU run at P that a rank
    # does for its shard only: the evaluation order and the schedule
    def dev_ms(fn, reps=3):
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        return float(np.median(ts))
    inv = torch.ones(gaN.P, dtype=torch.uint8, device=dev)
    lr = torch.empty(gaN.P, dtype=torch.int32, device=dev)
    lc = torch.empty(1, dtype=torch.int32, device=dev)
    res["order_ms_all_P"] = dev_ms(lambda: D.order(gaN.P, 0, inv, gaN.lineage_frames, True, lr, lc, gaN.ws))
    res["order_ms_shard"] = dev_ms(lambda: D.order(S, 0, inv, gaN.lineage_frames, True, lr[:S], lc, gaN.ws))
    res["schedule_ms_all_P"] = dev_ms(lambda: D.schedule("selfplay", gaN.P, gaN.n_games, 0, gaN.hof_fitness,
                                                        gaN.hof_n, gaN.seed, gaN.generation + 1, dev))
    res["schedule_ms_shard"] = dev_ms(lambda: D.schedule("selfplay", S, gaN.n_games, 0, gaN.hof_fitness,
                                                        gaN.hof_n, gaN.seed, gaN.generation + 1, dev))
    repl1 = float(np.median([w - e for w, e, _ in t1]))
    # a rank at N pays the one-GPU generation's non-evaluation time plus what
    # its P = N x 65 536 ops (sharded variation) cost beyond the same ops at
    # 65 536; its shard-sized work (evaluation prep, order, scatter) as at N = 1
    replN = repl1 + max(0.0, ops["replicated_critical_ms"] - ops1["replicated_critical_ms"])
    res["replicated_ms_pN_wall"] = float(np.median([w - e for w, e in zip(walls, evals)]))
    # the one-GPU wall at P less the P-row record preparation a rank does not
    # pay (it prepares its shard's rows, as at N = 1): against replicated_ms_pN
    res["replicated_ms_pN_wall_less_prep"] = (res["replicated_ms_pN_wall"] - res["genome_prep_ms_all_P"]
                                              + res["genome_prep_ms_shard"])
    res["replicated_ms_pN_wall_less_row_work"] = (res["replicated_ms_pN_wall_less_prep"]
                                                  - res["order_ms_all_P"] + res["order_ms_shard"]
                                                  - res["schedule_ms_all_P"] + res["schedule_ms_shard"])
    shard_max = float(np.median([max(x[0] for x in s) for s in shards]))
    shard_mean = float(np.median([float(np.mean([x[0] for x in s])) for s in shards]))
    steps_n = float(np.median([sum(x[1] for x in s) for s in shards]))  # all ranks' stepped env-steps
    allgather = 0.03 + N * S * 12 / 1e12 * 1e3  # ms
    t_n = shard_max + replN + allgather
    replN_s = repl1 + max(0.0, ops["replicated_critical_ms_streams"] - ops1["replicated_critical_ms_streams"])
    t_n_s = shard_max + replN_s + allgather
    t_1 = float(np.median(res["p65536_wall_ms"]))  # the measured one-GPU generation
    steps_1 = float(np.median(res["p65536_steps"]))
    ps_1 = float(np.median(res["p65536_ps_per_step"]))
    ps_n = float(np.median([float(np.mean([x[0] * 1e9 / x[1] for x in s])) for s in shards]))
    res.update({"replicated_ms_p65536": repl1, "replicated_ms_pN": replN, "shard_eval_ms_max": shard_max,
                "shard_eval_ms_mean": shard_mean, "straggler_factor": shard_max / shard_mean,
                "one_gpu_eval_ms": float(np.median(res["p65536_eval_ms"])),
                "steps_per_shard_pN": steps_n / N, "steps_one_gpu": steps_1,
                "ps_per_step_shard_pN": ps_n, "ps_per_step_one_gpu": ps_1,
                "allgather_ms_model": allgather, "t1_ms": t_1, "tN_ms": t_n, "projected_efficiency": t_1 / t_n,
                "projected_speedup": N * t_1 / t_n,
                # the same with the critical path of the code's stream structure
                "replicated_ms_pN_streams": replN_s, "tN_ms_streams": t_n_s,
                "projected_efficiency_streams": t_1 / t_n_s,
                "projected_env_steps_per_s_N": steps_n / (t_n / 1e3),
                "env_steps_per_s_1": steps_1 / (t_1 / 1e3),
                "projected_efficiency_env_steps": (steps_n / t_n) / (N * steps_1 / t_1)})
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
