# round 2, session 4, call e2: k_service micro-optimisations (one-player CPU
# paddle as a branch, certificate thresholds moved once per pass) A/B
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r2_e2}; mkdir -p $OUT
timeout -k 10 400 python -u tools/sweep.py --libs variants/lib_svcbase.so,variants/lib_svccert.so,variants/lib_svcphys.so,variants/lib_svcbase.so,variants/lib_svccert.so,variants/lib_svcphys.so --lanes 8 --reps 3 --kernel split > $OUT/sweep.log 2>&1 || exit 1
echo done > $OUT/ok
