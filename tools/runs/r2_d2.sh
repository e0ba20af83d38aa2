# round 2, session 4, call d2: k_service per-wave frame rates (timeline build)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_d2; mkdir -p $OUT
PONG_GA_LIB=variants/lib_timeline.so timeout -k 10 300 python -u tools/timeline.py --lanes 8 --out $OUT/timeline.npz > $OUT/timeline.log 2>&1 || exit 1
echo done > $OUT/ok
