# round 3, call g4: how often a wave-frame takes each rare path (probe
# build), then the g3 steps (GPU suite, generation profiles, wide f32/f64)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_g4}; mkdir -p $OUT
timeout -k 10 300 python -u tools/sweep.py --libs variants/lib_pathprobe.so --lanes 8 --reps 1 --kernel split > $OUT/pathprobe.log 2>&1 || exit 1
RUN=r3_g4 bash tools/runs/r3_g3.sh || exit 1
echo done > $OUT/ok
