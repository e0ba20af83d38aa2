# round 3, call c2: game-start cost probe (PG_START_PROBE: shader cycles of the
# waves' game-start blocks vs their total), with and without the serve jump
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_c2}; mkdir -p $OUT
timeout -k 10 300 python -u tools/sweep.py --libs variants/lib_probe_nojump.so,variants/lib_probe.so --lanes 8 --reps 2 --kernel split > $OUT/sweep.log 2>&1 || exit 1
echo done > $OUT/ok
