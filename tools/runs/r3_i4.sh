# round 3, call i4: the rally search opened at a point's 8th return (64-frame
# first span) -- parity, same-box A/B against the h2 library, the bench
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_i4}; mkdir -p $OUT
B=variants/base_h2.so; N=neuro-genetic-pong-self-play_amd/libpong_ga.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hard_cases.py tests/test_gpu_evolve.py tests/test_gpu_generation.py tests/test_gpu_dropin.py tests/test_gpu_wide.py -x -q --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1 || exit 1
timeout -k 10 900 python -u tools/sweep.py --libs $B,$N,$B,$N,$B,$N --lanes 8 --reps 5 --kernel split > $OUT/sweep.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
PONG_GA_LIB=$B timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_base.json 2> $OUT/bench_base.err || exit 1
echo done > $OUT/ok
