# round 2, session 4, call d9: frame cost without f64 re-decisions (timing-only
# ablation builds): k_service vs k_inwave
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_d9; mkdir -p $OUT
timeout -k 10 400 python -u tools/sweep.py --libs variants/lib_svcabl.so,variants/lib_inwaveabl.so,variants/lib_svcabl.so,variants/lib_inwaveabl.so --lanes 8 --reps 3 --kernel split > $OUT/sweep.log 2>&1 || exit 1
echo done > $OUT/ok
