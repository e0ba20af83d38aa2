# round 2, session 3, call 6: which half of the genome_rows / n_active change costs k_service its 14 %
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_b6; mkdir -p $OUT
V=variants
timeout -k 10 600 python -u tools/sweep.py --libs $V/lib_svcmin2.so,$V/lib_xf.so,$V/lib_xg.so,$V/lib_xh.so,$V/lib_xb.so --lanes 8 --reps 3 --kernel split > $OUT/sweep.log 2>&1 || exit 1
echo done > $OUT/ok
