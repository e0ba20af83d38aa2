# round 2, session 3, call 3: k_staged phase timing (profile build), and the
# k_service regression A/B: round-1 tree vs current (min build), cheap service
# sigmoid, no f64 re-decisions.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_b3; mkdir -p $OUT
L=neuro-genetic-pong-self-play_amd/libpong_ga.so
PONG_GA_LIB=$(pwd)/variants/lib_prof.so timeout -k 10 200 python -u tools/staged_probe.py > $OUT/staged_probe.json 2> $OUT/staged_probe.err || exit 1
timeout -k 10 400 python -u tools/sweep.py --libs $L,variants/lib_svcmin.so,variants/lib_svcfast.so,variants/lib_svcnoskip.so,$L --lanes 8 --reps 3 --kernel split > $OUT/sweep.log 2>&1 || exit 1
(cd variants/old && timeout -k 10 200 python -u tools/sweep.py --lanes 8 --reps 3 --kernel split) > $OUT/sweep_old.log 2>&1 || exit 1
echo done > $OUT/ok
