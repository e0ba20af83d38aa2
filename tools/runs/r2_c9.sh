# round 2, session 4, call 9: the committed k_wide (non-temporal tile-major
# stream) at BASELINE config 5 -- GPU suite, bench --config wide, rocprof
# kernel stats, PMC FETCH/WRITE passes
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_c9; mkdir -p $OUT
ROOT=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --config wide > $OUT/bench_wide.json 2> $OUT/bench_wide.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof_wide -o kt -- python3 bench.py --config wide --no-cpu-baseline > $OUT/prof_wide.json 2> $OUT/prof_wide.err || exit 1
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_$ctr -o pmc -- python3 bench.py --config wide --no-cpu-baseline > $OUT/pmc_$ctr.json 2> $OUT/pmc_$ctr.err || exit 1
done
python3 tools/pmc_traffic.py $OUT $OUT/pmc_traffic_wide.json k_wide > $OUT/pmc.log 2>&1 || exit 1
echo done > $OUT/ok
