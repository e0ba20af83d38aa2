#!/usr/bin/env python3
"""Summarise tools/pmc_resident.sh output: per-env-step instruction counts and wave-cycle shares."""
import collections
import csv
import json
import sys

for tag in sys.argv[1:]:
    vals = collections.defaultdict(list)
    steps = None
    for p in ("p1", "p2"):
        for r in csv.DictReader(open(f"{tag}/{p}/pmc_counter_collection.csv")):
            if any(k in r["Kernel_Name"] for k in ("k_resident", "k_split", "k_service")):
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
        try:
            js = json.loads(open(f"{tag}/{p}.out").read().strip().splitlines()[-1])
            steps = js["env_steps"]
            episode = steps + js.get("rally_frames", 0) + js.get("hidden_frames", 0)
        except Exception:
            pass
    d = {k: v[-1] for k, v in vals.items()}
    wc = d["SQ_WAVE_CYCLES"]
    print(tag, "steps", steps)
    print("  per env-step: VALU %.1f SALU %.1f BRANCH %.1f LDS %.2f VMEM_RD %.2f VMEM_WR %.2f" % tuple(
        d[k] / steps for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR")))
    print("  wave-cycle shares: wait_any %.2f wait_inst_any %.2f active_any %.2f active_valu %.2f active_sca %.2f" % tuple(
        d[k] / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA")))
    print("  busy cycles %.3g, wave-cycles per step %.1f" % (d["SQ_BUSY_CYCLES"], wc / steps))
    print("  per episode frame (%d): VALU %.1f SALU %.1f" % (episode, d["SQ_INSTS_VALU"] / episode,
                                                             d["SQ_INSTS_SALU"] / episode))
