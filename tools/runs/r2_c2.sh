# round 2, session 4, call 2: k_wide streaming W2 from tile-major per-block
# copies straight into registers (no LDS tile, no per-tile barriers) --
# wide GPU tests, A/B sweep vs the previous k_wide at pop 4096, ring depth 3,
# no scheduling fence, streaming-only
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_c2; mkdir -p $OUT
L=neuro-genetic-pong-self-play_amd/libpong_ga.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_wide.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/sweep.py --libs variants/lib_head.so,$L,variants/lib_wd3.so,variants/lib_wnofence.so,variants/lib_wnocomp.so,$L --lanes 0 --reps 2 --kernel wide --shape 6,512,512,3 --dtype f32 --pop 4096 > $OUT/sweep_wide.log 2>&1 || exit 1
echo done > $OUT/ok
