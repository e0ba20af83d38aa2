# round 4, the final library, call 1 of 2: the whole -m gpu suite, smoke(), and
# the FETCH_SIZE / WRITE_SIZE PMC passes of every bench workload (the headline,
# --horizon 1000, --schedule reference, --dist init, the wide config), each
# reduced by tools/pmc_traffic.py to HBM bytes per launch, hash-matched to the
# library (copied into profiles/r04/ afterwards, so call 2's bench lines report them)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r4_final1}; mkdir -p $OUT; ROOT=$(pwd)
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
pmc pmc_horizon k_service --steps 1 --warmup 1 --horizon 1000 || exit 1
pmc pmc_reference k_service --steps 1 --warmup 1 --schedule reference || exit 1
pmc pmc_init k_service --steps 1 --warmup 1 --dist init || exit 1
pmc pmc_wide k_wide --config wide || exit 1
echo done > $OUT/ok
