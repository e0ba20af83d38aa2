#!/usr/bin/env python3
"""Per-dispatch durations of the evaluation kernel from a rocprofv3
--kernel-trace CSV, split into the warm-up and timed launches of bench.py,
for comparison with bench.py's HIP-event kernel_ms_per_launch.
usage: python tools/trace_summary.py gpurun_out/TAG/prof/kt_kernel_trace.csv WARMUP [out.json]
"""
import csv
import json
import sys


def main():
    path, warm = sys.argv[1], int(sys.argv[2])
    rows = [r for r in csv.DictReader(open(path)) if "k_service" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    timed = ms[warm:]
    res = {"kernel": rows[0]["Kernel_Name"] if rows else None, "launches_ms": ms,
           "timed_mean_ms": sum(timed) / max(len(timed), 1), "warmup": warm}
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as fh:
            json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
