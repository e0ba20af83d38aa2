# round 3, call i7: ABI 7 prep modes (genome lane records + self-play
# schedule made during the hall-of-fame scan; counters zeroed by the prep
# kernel) -- the whole -m gpu suite, bench with / without the early prep
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_i7}; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
PG_NO_EARLY_PREP=1 timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_noearly.json 2> $OUT/bench_noearly.err || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench2.json 2> $OUT/bench2.err || exit 1
PG_NO_EARLY_PREP=1 timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_noearly2.json 2> $OUT/bench_noearly2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof -o kt -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
echo done > $OUT/ok
