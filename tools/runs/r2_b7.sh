# round 2, session 3, call 7: the uniform loop-bound fix -- full GPU suite
# (incl. k_staged), smoke, sweep (split vs staged), bench + rocprof + PMC passes.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_b7; mkdir -p $OUT
ROOT=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/sweep.py --lanes 8 --reps 3 --kernel split > $OUT/sweep_split.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/sweep.py --lanes 8 --reps 3 --kernel staged > $OUT/sweep_staged.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_$ctr -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_$ctr.json 2> $OUT/pmc_$ctr.err || exit 1
done
echo done > $OUT/ok
