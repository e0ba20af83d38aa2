# round 2, session 3, call 2: first run of k_staged -- its GPU tests, then the
# bench workload's single-launch sweep (split vs staged) and the bench with staged.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_b2; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_staged.py -x -v --timeout 120 --timeout-method thread > $OUT/staged_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/sweep.py --lanes 8 --reps 3 --kernel split > $OUT/sweep_split.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/sweep.py --lanes 8 --reps 3 --kernel staged > $OUT/sweep_staged.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --kernel staged > $OUT/bench_staged.json 2> $OUT/bench_staged.err || exit 1
echo done > $OUT/ok
