#!/bin/bash
# GPU-box session for the wide kernel: its parity tests, then probe timings.
# usage: tools/gpu_wide.sh TAG [probe pops...]
TAG=${1:-wide}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/tests.log" 2>&1
rc=$?; echo "wide tests exit=$rc" >> "$OUT/summary.txt"; [ $rc -ne 0 ] && exit $rc
for pop in "$@"; do
  timeout -k 10 300 python -u tools/wide_probe.py $pop >> "$OUT/probe.log" 2>&1
  rc=$?; echo "probe $pop exit=$rc" >> "$OUT/summary.txt"; [ $rc -ne 0 ] && exit $rc
done
exit 0
