# round 2, session 4, call i1: serve-and-play (PG_SVC_PLAY): one small
# evaluation first (stop on any error), the parity-critical tests through the
# variant, then the A/B sweep
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r2_i1}; mkdir -p $OUT
PONG_GA_LIB=variants/lib_svcplay.so timeout -k 10 120 python -u tools/sweep.py --one --lane=8 --reps 1 --pop 1024 --kernel split > $OUT/small.log 2>&1 || exit 1
grep -q env_steps $OUT/small.log || exit 1
PONG_GA_LIB=variants/lib_svcplay.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "near_saturation or episode_traces or hard" > $OUT/parity.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/sweep.py --libs variants/lib_svcbase.so,variants/lib_svcplay.so,variants/lib_svcbase.so,variants/lib_svcplay.so --lanes 8 --reps 3 --kernel split > $OUT/sweep.log 2>&1 || exit 1
echo done > $OUT/ok
