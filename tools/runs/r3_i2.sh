# round 3, call i2: per-game timeline of the bench's own evaluation launch at
# generations 12 and 24, with the length predictors' correlations
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_i2}; mkdir -p $OUT
PONG_GA_LIB=variants/timeline.so timeout -k 10 300 python -u tools/timeline_ga.py --gens 12 --out $OUT/tl12.npz > $OUT/timeline_ga12.log 2>&1 || exit 1
PONG_GA_LIB=variants/timeline.so timeout -k 10 300 python -u tools/timeline_ga.py --gens 24 --out $OUT/tl24.npz > $OUT/timeline_ga24.log 2>&1 || exit 1
echo done > $OUT/ok
