# round 2, session 4, call 3: k_wide phase split (shader-clock stamps build)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_c3; mkdir -p $OUT
timeout -k 10 300 python -u tools/sweep.py --libs variants/lib_wstamps.so --lanes 0 --reps 1 --kernel wide --shape 6,512,512,3 --dtype f32 --pop 4096 > $OUT/sweep_stamps.log 2>&1 || exit 1
echo done > $OUT/ok
