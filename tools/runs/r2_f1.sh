# round 2, session 4, call f1: profiles of the committed build -- GPU suite,
# smoke, bench (with the CPU baseline), rocprof kernel stats, PMC FETCH/WRITE
# and SQ counters of k_service; config 5 bench, rocprof and PMC of k_wide
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_f1; mkdir -p $OUT
ROOT=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_$ctr -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_$ctr.json 2> $OUT/pmc_$ctr.err || exit 1
done
python3 tools/pmc_traffic.py $OUT $OUT/pmc_traffic.json k_service > $OUT/pmc.log 2>&1 || exit 1
bash tools/pmc_resident.sh r2_f1/sq 8 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_FLAT SQ_INSTS_VALU_CVT --kernel-trace --output-format csv -d $ROOT/$OUT/sq/p3 -o pmc -- python3 tools/sweep.py --one --lane=8 --reps 1 > $OUT/sq/p3.out 2> $OUT/sq/p3.err || exit 1
timeout -k 10 400 python -u bench.py --config wide > $OUT/bench_wide.json 2> $OUT/bench_wide.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof_wide -o kt -- python3 bench.py --config wide --no-cpu-baseline > $OUT/prof_wide.json 2> $OUT/prof_wide.err || exit 1
mkdir -p $OUT/w
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $ROOT/$OUT/w/pmc_$ctr -o pmc -- python3 bench.py --config wide --no-cpu-baseline > $OUT/w/pmc_$ctr.json 2> $OUT/w/pmc_$ctr.err || exit 1
done
python3 tools/pmc_traffic.py $OUT/w $OUT/pmc_traffic_wide.json k_wide > $OUT/pmc_wide.log 2>&1 || exit 1
echo done > $OUT/ok
