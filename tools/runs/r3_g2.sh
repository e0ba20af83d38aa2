# round 3, call g2: section timing of the in-wave k_service (probe build) and
# a longer A/B of base / certify / in-wave
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_g2}; mkdir -p $OUT
B=neuro-genetic-pong-self-play_amd/libpong_ga.so
timeout -k 10 300 python -u tools/sweep.py --libs variants/lib_inwave_sp.so --lanes 8 --reps 2 --kernel split > $OUT/probe.log 2>&1 || exit 1
timeout -k 10 900 python -u tools/sweep.py --libs $B,variants/lib_cert.so,variants/lib_inwave.so,$B,variants/lib_cert.so,variants/lib_inwave.so,$B,variants/lib_cert.so,variants/lib_inwave.so --lanes 8 --reps 5 --kernel split > $OUT/sweep.log 2>&1 || exit 1
echo done > $OUT/ok
