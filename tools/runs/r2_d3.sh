# round 2, session 4, call d3: k_inwave (every wave plays, f64 cascade in-wave)
# vs k_service -- A/B sweep, inwave timeline
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_d3; mkdir -p $OUT
L=neuro-genetic-pong-self-play_amd/libpong_ga.so
timeout -k 10 400 python -u tools/sweep.py --libs variants/lib_svcmin.so,variants/lib_inwave.so,variants/lib_svcmin.so,variants/lib_inwave.so --lanes 8 --reps 3 --kernel split > $OUT/sweep.log 2>&1 || exit 1
echo done > $OUT/ok
