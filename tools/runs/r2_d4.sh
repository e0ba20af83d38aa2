# round 2, session 4, call d4: k_inwave after the slot-index fix -- one small
# evaluation first (stop on any error), then the A/B sweep
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r2_d4}; mkdir -p $OUT
PONG_GA_LIB=variants/lib_inwave.so timeout -k 10 120 python -u tools/sweep.py --one --lane=8 --reps 1 --pop 1024 --kernel split > $OUT/small.log 2>&1 || exit 1
grep -q env_steps $OUT/small.log || exit 1
timeout -k 10 400 python -u tools/sweep.py --libs variants/lib_svcmin.so,variants/lib_inwave.so,variants/lib_svcmin.so,variants/lib_inwave.so --lanes 8 --reps 3 --kernel split > $OUT/sweep.log 2>&1 || exit 1
echo done > $OUT/ok
