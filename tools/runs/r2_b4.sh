# round 2, session 3, call 4: k_staged after the overlapped start pipeline
# (phase probe + sweep), k_service with the compact service sigmoid, round-1 tree.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_b4; mkdir -p $OUT
PONG_GA_LIB=$(pwd)/variants/lib_prof.so timeout -k 10 200 python -u tools/staged_probe.py > $OUT/staged_probe.json 2> $OUT/staged_probe.err || exit 1
timeout -k 10 400 python -u tools/sweep.py --libs variants/lib_stg2.so --lanes 8 --reps 3 --kernel staged > $OUT/sweep_staged.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/sweep.py --libs variants/lib_svcmin2.so --lanes 8 --reps 3 --kernel split > $OUT/sweep_split.log 2>&1 || exit 1
(cd variants/old && timeout -k 10 200 python -u tools/sweep.py --lanes 8 --reps 3 --kernel split) > $OUT/sweep_old.log 2>&1 || exit 1
echo done > $OUT/ok
