#!/usr/bin/env python3
"""Table of the bench lines an A/B call wrote (gpurun_out/<tag>/<mode>_<variant>_<rep>.json):
per line the stepped env-steps/s, ms per step, the kernel's ms per launch (HIP
events), roofline.frac and the cascade's counters.  The call's lib_sha.txt
(which library each variant was) and its script's header comment go on top.

    python tools/ab_summary.py gpurun_out/r6_c4 [tools/runs/r6_c4.sh] > profiles/r06/ab_....txt
"""
import glob
import json
import os
import sys


def main(d, script=None):
    if script and os.path.exists(script):
        for line in open(script):
            if line.startswith("#"):
                print(line.rstrip())
            elif line.strip():
                break
    sha = os.path.join(d, "lib_sha.txt")
    if os.path.exists(sha):
        print("# libraries:")
        for line in open(sha):
            print("#  ", line.rstrip())
    cols = ("file", "value_e9", "ms_step", "kernel_ms", "frac", "fail/fwd", "in_wave", "f64_cert")
    print("%-28s %9s %8s %9s %6s %9s %7s %8s" % cols)
    for f in sorted(glob.glob(os.path.join(d, "*.json"))):
        try:
            j = json.load(open(f))
        except (ValueError, OSError):
            continue
        if "value" not in j:
            continue
        c, r = j.get("config", {}), j.get("roofline", {})
        ms = r.get("kernel_ms_per_launch", r.get("ms_per_launch"))
        print("%-28s %9.4f %8.3f %9.4f %6.3f %9.6f %7.3f %8.3f" % (
            os.path.basename(f), j["value"] / 1e9, j["ms_per_step"], ms or float("nan"), r.get("frac", float("nan")),
            c.get("certificate_failures_per_forward", float("nan")), c.get("failures_decided_in_wave", float("nan")),
            c.get("failures_decided_by_f64_certificate", float("nan"))))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
