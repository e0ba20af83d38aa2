# round 2, session 3, call 5: bisect the k_service slowdown since round 1
# (hard-log code, genome_rows/n_active indirection, certify's underflow rule).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_b5; mkdir -p $OUT
V=variants
timeout -k 10 600 python -u tools/sweep.py --libs $V/lib_svcmin2.so,$V/lib_xa.so,$V/lib_xb.so,$V/lib_xc.so,$V/lib_xd.so,$V/lib_xe.so,$V/lib_svcmin2.so --lanes 8 --reps 3 --kernel split > $OUT/sweep.log 2>&1 || exit 1
(cd variants/old && timeout -k 10 200 python -u tools/sweep.py --lanes 8 --reps 3 --kernel split) > $OUT/sweep_old.log 2>&1 || exit 1
echo done > $OUT/ok
