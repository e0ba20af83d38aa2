# round 3, call e1: next-game prefetch (the work claim and schedule loads a
# game ahead) and two-accumulator W2 sums -- parity first, then A/B sweeps
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_e1}; mkdir -p $OUT
timeout -k 10 120 python -u tools/sweep.py --one --lane=8 --reps 1 --pop 1024 --kernel split > $OUT/small.log 2>&1 || exit 1
grep -q env_steps $OUT/small.log || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hard_cases.py tests/test_gpu_evolve.py -x -q --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1 || exit 1
PONG_GA_LIB=variants/lib_w2split.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "near_saturation or episode_traces or layouts" > $OUT/parity_w2.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/sweep.py --libs variants/lib_base.so,neuro-genetic-pong-self-play_amd/libpong_ga.so,variants/lib_w2split.so,variants/lib_base.so,neuro-genetic-pong-self-play_amd/libpong_ga.so,variants/lib_w2split.so --lanes 8 --reps 3 --kernel split > $OUT/sweep.log 2>&1 || exit 1
echo done > $OUT/ok
