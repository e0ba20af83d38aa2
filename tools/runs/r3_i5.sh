# round 3, call i5: frame trims 4 (untraced k_service instance, per-network
# certificate constants, Pong::step's face event) -- the whole -m gpu suite,
# same-box A/B against the i4 library (sweep + bench)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_i5}; mkdir -p $OUT
B=variants/base_i4.so; N=neuro-genetic-pong-self-play_amd/libpong_ga.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 900 python -u tools/sweep.py --libs $B,$N,$B,$N,$B,$N --lanes 8 --reps 5 --kernel split > $OUT/sweep.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
PONG_GA_LIB=$B timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_base.json 2> $OUT/bench_base.err || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench2.json 2> $OUT/bench2.err || exit 1
echo done > $OUT/ok
