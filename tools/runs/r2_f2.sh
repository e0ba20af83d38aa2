# round 2, session 4, call f2: the bench lines against the refreshed
# profiles/r02 PMC summaries (so every roofline field reproduces from profiles/)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r2_f2}; mkdir -p $OUT
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 400 python -u bench.py --config wide > $OUT/bench_wide.json 2> $OUT/bench_wide.err || exit 1
echo done > $OUT/ok
