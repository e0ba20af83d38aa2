# round 2, session 3, call 10: k_staged with one sync word (no polling scan/sleep)
# and the decision-independent bookkeeping moved before the wait
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_b10; mkdir -p $OUT
PONG_GA_LIB=$(pwd)/variants/lib_stg3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_staged.py -x -v --timeout 120 --timeout-method thread > $OUT/staged_tests.log 2>&1 || exit 1
PONG_GA_LIB=$(pwd)/variants/lib_prof.so timeout -k 10 200 python -u tools/staged_probe.py > $OUT/staged_probe.json 2> $OUT/staged_probe.err || exit 1
timeout -k 10 300 python -u tools/sweep.py --libs variants/lib_stg3.so --lanes 8 --reps 3 --kernel staged > $OUT/sweep.log 2>&1 || exit 1
echo done > $OUT/ok
