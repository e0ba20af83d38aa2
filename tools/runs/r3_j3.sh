# round 3, call j3: lane layouts of the split kernel on today's frame path
# (L = 8 / 16 / 32 games per wave of 8 / 4 / 2), same box, alternating
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_j3}; mkdir -p $OUT
timeout -k 10 500 python3 -u tools/sweep.py --lanes 8,16,32,8,16,32,8,16 --reps 4 > $OUT/sweep_lanes.log 2>&1 || exit 1
echo done > $OUT/ok
