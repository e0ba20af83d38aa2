# round 3, call i1: per-game timeline of the bench's own evaluation launch
# (after 12 GA generations), length-ordered queue vs plain order
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_i1}; mkdir -p $OUT
PONG_GA_LIB=variants/timeline.so timeout -k 10 300 python -u tools/timeline_ga.py --gens 12 > $OUT/timeline_ga.log 2>&1 || exit 1
PONG_GA_LIB=variants/timeline.so timeout -k 10 300 python -u tools/timeline_ga.py --gens 12 --no-order > $OUT/timeline_ga_noorder.log 2>&1 || exit 1
echo done > $OUT/ok
