# round 4, the final library: the whole -m gpu suite, smoke(); the FETCH/WRITE
# PMC passes of the headline bench, of its --horizon 1000, --schedule reference
# and --dist init runs and of the wide
# bench (written into profiles/r04/ on the box first, so each bench line below
# reports its counter traffic); the driver's bench command, the secondary runs
# (--horizon 1000, --schedule reference, --dist init), the wide line; a rocprof
# kernel trace of the headline; the SQ counters of k_service
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r4_final}; mkdir -p $OUT profiles/r04; ROOT=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
pmc() {  # tag, kernel, bench args...
  local tag=$1 kern=$2; shift 2
  mkdir -p $OUT/$tag
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 400 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $ROOT/$OUT/$tag/pmc_$ctr -o pmc -- python3 $ROOT/bench.py --no-cpu-baseline "$@" > $OUT/$tag/pmc_$ctr.json 2> $OUT/$tag/pmc_$ctr.err || return 1
  done
  python3 tools/pmc_traffic.py $OUT/$tag $OUT/$tag/pmc_traffic.json $kern > $OUT/$tag/pmc.log 2>&1 || return 1
}
pmc pmc_head k_service --steps 2 --warmup 1 || exit 1
cp $OUT/pmc_head/pmc_traffic.json profiles/r04/pmc_traffic.json
pmc pmc_horizon k_service --steps 1 --warmup 1 --horizon 1000 || exit 1
cp $OUT/pmc_horizon/pmc_traffic.json profiles/r04/pmc_traffic_horizon1000.json
pmc pmc_reference k_service --steps 1 --warmup 1 --schedule reference || exit 1
cp $OUT/pmc_reference/pmc_traffic.json profiles/r04/pmc_traffic_reference.json
pmc pmc_init k_service --steps 1 --warmup 1 --dist init || exit 1
cp $OUT/pmc_init/pmc_traffic.json profiles/r04/pmc_traffic_init.json
pmc pmc_wide k_wide --config wide || exit 1
cp $OUT/pmc_wide/pmc_traffic.json profiles/r04/pmc_traffic_wide.json
timeout -k 10 600 python3 -u tools/scale_model.py 8 4 > $OUT/scale_model.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --horizon 1000 > $OUT/bench_horizon.json 2> $OUT/bench_horizon.err || exit 1
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --schedule reference > $OUT/bench_reference.json 2> $OUT/bench_reference.err || exit 1
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --dist init > $OUT/bench_init.json 2> $OUT/bench_init.err || exit 1
timeout -k 10 600 python3 -u bench.py --config wide --gpus 1 --steps 2 --warmup 1 > $OUT/bench_wide.json 2> $OUT/bench_wide.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof -o kt -- python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
bash tools/pmc_sq.sh ${RUN:-r4_final}/sq 8 || exit 1
python3 tools/pmc_summary.py $OUT/sq > $OUT/sq_summary.txt 2>&1 || exit 1
echo done > $OUT/ok
