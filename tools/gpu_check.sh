#!/bin/bash
# GPU-box session: parity tests, bench, rocprof kernel-trace stats.  Each GPU
# step has its own time limit; a fault/abort/timeout stops the script.
# usage: tools/gpu_check.sh TAG [bench args...]
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
fatal() { case "$1" in 124|134|137|139) echo "fatal exit $1 in $2" >> "$OUT/summary.txt"; exit "$1";; esac; }
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout=400 -p no:cacheprovider > "$OUT/tests.log" 2>&1
rc=$?; echo "tests exit=$rc" >> "$OUT/summary.txt"; fatal $rc tests
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke exit=$rc" >> "$OUT/summary.txt"; fatal $rc smoke
timeout -k 10 400 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench exit=$rc" >> "$OUT/summary.txt"; fatal $rc bench
ROOT=$(pwd)
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o kt --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline "$@" > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
rc=$?; echo "rocprof exit=$rc" >> "$OUT/summary.txt"; fatal $rc rocprof
if [ -n "$PMC" ]; then
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 400 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$ROOT/$OUT/pmc_$ctr" -o pmc -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline "$@" > "$OUT/pmc_$ctr.json" 2> "$OUT/pmc_$ctr.err"
    rc=$?; echo "pmc $ctr exit=$rc" >> "$OUT/summary.txt"; fatal $rc pmc
  done
fi
exit 0
