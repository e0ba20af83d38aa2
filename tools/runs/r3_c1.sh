# round 3, call c1: the serve-delay jump in k_service -- parity suite, then
# a same-box A/B against the no-jump variant on the bench workload
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_c1}; mkdir -p $OUT
timeout -k 10 120 python -u tools/sweep.py --one --lane=8 --reps 1 --pop 1024 --kernel split > $OUT/small.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hard_cases.py -x -q --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/sweep.py --libs variants/lib_nojump.so,neuro-genetic-pong-self-play_amd/libpong_ga.so,variants/lib_nojump.so,neuro-genetic-pong-self-play_amd/libpong_ga.so --lanes 8 --reps 3 --kernel split > $OUT/sweep.log 2>&1 || exit 1
echo done > $OUT/ok
