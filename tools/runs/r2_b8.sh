# round 2, session 3, call 8: k_service micro-optimisations (left-network x-flip
# folded into its weights, branchy physics for face crossings, no per-frame NaN
# test, scripted/trace branches) -- parity suite, then A/B sweep vs the previous build.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_b8; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
L=neuro-genetic-pong-self-play_amd/libpong_ga.so
timeout -k 10 600 python -u tools/sweep.py --libs variants/lib_head.so,$L,variants/lib_head.so,$L --lanes 8 --reps 3 --kernel split > $OUT/sweep.log 2>&1 || exit 1
echo done > $OUT/ok
