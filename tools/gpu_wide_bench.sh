#!/bin/bash
# GPU-box session: the whole -m gpu suite, the headline bench, then BASELINE
# config 5 (wide MLP) bench + rocprof kernel trace + PMC traffic passes.
# usage: tools/gpu_wide_bench.sh TAG
TAG=${1:-wb}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
ROOT=$(pwd)
export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal exit $1 in $2" >> "$OUT/summary.txt"; exit "$1";; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > "$OUT/tests.log" 2>&1
fatal $? tests
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
fatal $? bench
timeout -k 10 400 python bench.py --config wide > "$OUT/bench_wide.json" 2> "$OUT/bench_wide.err"
fatal $? bench_wide
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof_wide" -o kt --output-format csv -- python3 "$ROOT/bench.py" --config wide --no-cpu-baseline > "$OUT/prof_wide.json" 2> "$OUT/prof_wide.err"
fatal $? rocprof_wide
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$ROOT/$OUT/pmc_$ctr" -o pmc -- python3 "$ROOT/bench.py" --config wide --no-cpu-baseline > "$OUT/pmc_$ctr.json" 2> "$OUT/pmc_$ctr.err"
  fatal $? pmc_$ctr
done
echo done >> "$OUT/summary.txt"
