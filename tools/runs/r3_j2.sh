# round 3, call j2: the solo phase (a wave's lone last game over all 64
# lanes) -- the whole -m gpu suite, a same-box A/B sweep against the build
# without it (-DPG_NO_SOLO), the driver's bench command on both, rocprof stats
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_j2}; mkdir -p $OUT; ROOT=$(pwd)
P=neuro-genetic-pong-self-play_amd/libpong_ga.so; V=variants/nosolo.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python3 -u tools/sweep.py --libs $V,$P,$V,$P,$V,$P --lanes 8 --reps 5 > $OUT/sweep.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
PONG_GA_LIB=$ROOT/$V timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_nosolo.json 2> $OUT/bench_nosolo.err || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench2.json 2> $OUT/bench2.err || exit 1
PONG_GA_LIB=$ROOT/$V timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_nosolo2.json 2> $OUT/bench_nosolo2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof -o kt -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
echo done > $OUT/ok
