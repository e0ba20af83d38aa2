# round 2, session 3, call 13: the committed build -- GPU suite, bench (with the
# CPU baseline), rocprof kernel stats, PMC FETCH/WRITE passes, SQ instruction
# counters of k_service (per-env-step VALU/SALU and the f32 mix)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_b13; mkdir -p $OUT
ROOT=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_$ctr -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_$ctr.json 2> $OUT/pmc_$ctr.err || exit 1
done
bash tools/pmc_resident.sh r2_b13/sq 8 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_FLAT SQ_INSTS_VALU_CVT --kernel-trace --output-format csv -d $ROOT/$OUT/sq/p3 -o pmc -- python3 tools/sweep.py --one --lane=8 --reps 1 > $OUT/sq/p3.out 2> $OUT/sq/p3.err || exit 1
echo done > $OUT/ok
