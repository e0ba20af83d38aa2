# round 3, call i3: timeline of the bench's generation-12 launch, with the
# 300 longest games' networks saved for a CPU replay (tools/long_games.py)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_i3}; mkdir -p $OUT
PONG_GA_LIB=variants/timeline.so timeout -k 10 300 python -u tools/timeline_ga.py --gens 12 --keep 300 --out $OUT/tl12.npz > $OUT/timeline_ga12.log 2>&1 || exit 1
echo done > $OUT/ok
