# round 3, call k1: the game-start and hidden-ball tests merged into one wave-uniform test; the scripted-left and 1-player tests read wave-uniform flags kept from the game starts
# -- the whole -m gpu suite, a same-box sweep A/B against the previous library
# (variants/base_k.so = build 3243d0d325969eb8), the driver's bench command on both
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_k1}; mkdir -p $OUT; ROOT=$(pwd)
P=neuro-genetic-pong-self-play_amd/libpong_ga.so; V=variants/base_k.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python3 -u tools/sweep.py --libs $V,$P,$V,$P,$V,$P --lanes 8 --reps 5 > $OUT/sweep.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
PONG_GA_LIB=$ROOT/$V timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_base.json 2> $OUT/bench_base.err || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench2.json 2> $OUT/bench2.err || exit 1
PONG_GA_LIB=$ROOT/$V timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_base2.json 2> $OUT/bench_base2.err || exit 1
echo done > $OUT/ok
