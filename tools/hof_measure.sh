#!/bin/bash
# GPU-box session: bench (default and 20 steps), GA phase profiles at 65k and
# 524k, hall-of-fame trace at 524k.  Each step time-limited; stops at the first failure.
# usage: tools/hof_measure.sh TAG
OUT=gpurun_out/${1:-hof}
mkdir -p "$OUT"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 3 > "$OUT/bench20.json" 2> "$OUT/bench20.err" &&
timeout -k 10 200 python tools/ga_profile.py 65536 8 > "$OUT/ga65k.log" 2>&1 &&
timeout -k 10 300 python tools/diag/hof_trace.py 524288 3 > "$OUT/trace_524k.txt" 2>&1 &&
timeout -k 10 300 python tools/ga_profile.py 524288 6 > "$OUT/ga524k.log" 2>&1
