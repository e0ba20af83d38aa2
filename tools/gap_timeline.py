#!/usr/bin/env python3
"""Device-idle intervals of bench.py generations from a rocprofv3 trace.

Reads ``<prefix>_kernel_trace.csv`` (and ``_memory_copy_trace.csv`` when
present), orders every device operation by start time and splits the run at
the evaluation launches (k_service / k_wide / k_general).  For each
generation (one evaluation launch to the next) it reports the evaluation
kernel's time, the other device operations' busy time, and the idle gaps
(no device operation running), listing the operations on either side of each
gap above ``--min-gap-us``.

usage: python tools/gap_timeline.py gpurun_out/TAG/prof/kt [--skip 2] [--min-gap-us 20] [--json out.json]
"""
import argparse
import csv
import json
import os

EVAL = ("k_service", "k_wide", "k_general", "k_resident", "k_staged")


def load(prefix):
    ops = []
    with open(prefix + "_kernel_trace.csv") as fh:
        for r in csv.DictReader(fh):
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    mc = prefix + "_memory_copy_trace.csv"
    if os.path.exists(mc):
        with open(mc) as fh:
            for r in csv.DictReader(fh):
                ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy:" + r["Direction"]))
    ops.sort()
    return ops


def short(name):
    n = name.split("(")[0]
    for k in EVAL:
        if k in n:
            return k
    return n.replace("void ", "").split("<")[0][-48:]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("prefix")
    p.add_argument("--skip", type=int, default=2, help="evaluation launches before the first timed one")
    p.add_argument("--min-gap-us", type=float, default=20.0)
    p.add_argument("--json", default=None)
    a = p.parse_args()
    ops = load(a.prefix)
    ev_idx = [i for i, o in enumerate(ops) if any(k in o[2] for k in EVAL)]
    gens = []
    for j in range(a.skip, len(ev_idx) - 1):
        i0, i1 = ev_idx[j], ev_idx[j + 1]
        seg = ops[i0:i1]
        t0, t_next = seg[0][0], ops[i1][0]
        kern = seg[0][1] - seg[0][0]
        busy, gaps, cur_end = 0, [], seg[0][1]
        prev = seg[0][2]
        for s, e, n in seg[1:]:
            if s > cur_end:
                gaps.append((s - cur_end, short(prev), short(n)))
            busy += max(0, e - max(s, cur_end))
            if e > cur_end:
                cur_end, prev = e, n
        if t_next > cur_end:
            gaps.append((t_next - cur_end, short(prev), short(ops[i1][2])))
        idle = sum(g[0] for g in gaps)
        gens.append({"gen": j, "period_ms": (t_next - t0) / 1e6, "eval_kernel_ms": kern / 1e6,
                     "other_busy_ms": busy / 1e6, "idle_ms": idle / 1e6, "n_ops": len(seg),
                     "gaps_us": [(round(g[0] / 1e3, 1), g[1], g[2]) for g in gaps if g[0] / 1e3 >= a.min_gap_us]})
    for g in gens:
        print(f"gen {g['gen']}: period {g['period_ms']:.3f} ms = eval {g['eval_kernel_ms']:.3f} + other busy "
              f"{g['other_busy_ms']:.3f} + idle {g['idle_ms']:.3f} ({g['n_ops']} ops)")
        for gap in g["gaps_us"]:
            print(f"    idle {gap[0]:8.1f} us  after {gap[1]}  before {gap[2]}")
    if gens:
        n = len(gens)
        summ = {k: sum(g[k] for g in gens) / n for k in ("period_ms", "eval_kernel_ms", "other_busy_ms", "idle_ms")}
        summ["non_kernel_ms"] = summ["period_ms"] - summ["eval_kernel_ms"]
        print("mean:", json.dumps(summ))
        if a.json:
            with open(a.json, "w") as fh:
                json.dump({"mean": summ, "generations": gens}, fh, indent=1)


if __name__ == "__main__":
    main()
