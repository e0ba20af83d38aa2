# round 2, session 4, call 1: k_service mailbox on LDS atomics (no flat ops),
# k_service split into two translation units -- GPU suite, A/B vs the
# previous build, SQ FLAT/VALU counters
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_c1; mkdir -p $OUT
ROOT=$(pwd)
L=neuro-genetic-pong-self-play_amd/libpong_ga.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/sweep.py --libs variants/lib_head.so,$L,variants/lib_head.so,$L --lanes 8 --reps 3 --kernel split > $OUT/sweep.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_FLAT SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SMEM --kernel-trace --output-format csv -d $ROOT/$OUT/sq -o pmc -- python3 tools/sweep.py --one --lane=8 --reps 1 > $OUT/sq.out 2> $OUT/sq.err || exit 1
echo done > $OUT/ok
