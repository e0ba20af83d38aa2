# round 2, session 4, call e4-5: k_wide W1 variants
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r2_e4}; mkdir -p $OUT
L=neuro-genetic-pong-self-play_amd/libpong_ga.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_wide.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/sweep.py --libs $L,variants/lib_wrows.so,$L,variants/lib_wrows.so --lanes 0 --reps 2 --kernel wide --shape 6,512,512,3 --dtype f32 --pop 4096 > $OUT/sweep_wide.log 2>&1 || exit 1
echo done > $OUT/ok
