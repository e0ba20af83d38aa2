# round 2, session 4, call 4-5: k_wide with uniform descriptors (no waterfall
# loops), W3 resident in LDS, quad-parallel layer 3, ring prologue before
# layer 1 -- wide GPU tests, A/B sweep at pop 4096, depth 3, phase stamps
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r2_c4}; mkdir -p $OUT
L=neuro-genetic-pong-self-play_amd/libpong_ga.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_wide.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/sweep.py --libs $L,variants/lib_wnt.so,variants/lib_ww1.so,variants/lib_wntw1.so,variants/lib_wntstamps.so,$L --lanes 0 --reps 2 --kernel wide --shape 6,512,512,3 --dtype f32 --pop 4096 > $OUT/sweep_wide.log 2>&1 || exit 1
echo done > $OUT/ok
