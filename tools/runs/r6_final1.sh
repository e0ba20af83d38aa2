# round 6, the final library, call 1 of 2: the whole -m gpu suite and smoke();
# the FETCH_SIZE / WRITE_SIZE PMC passes of every bench workload (reduced by
# tools/pmc_traffic.py, hash-matched to the library) copied into this box's
# profiles/r06/ so that the bench lines after them report roofline.traffic;
# the driver's bench command and the secondary lines (--horizon 1000,
# --schedule reference, --dist init).  Afterwards gpurun_out/<tag>/* is
# copied into profiles/r06/ (*_final.*).
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_final}
OUT=gpurun_out/$TAG; mkdir -p $OUT; ROOT=$(pwd)
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so > $OUT/lib_sha.txt
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
pmc() {  # tag, kernel, output name, bench args...
  local tag=$1 kern=$2 name=$3; shift 3
  mkdir -p $OUT/$tag
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 400 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $ROOT/$OUT/$tag/pmc_$ctr -o pmc -- python3 $ROOT/bench.py --no-cpu-baseline "$@" > $OUT/$tag/pmc_$ctr.json 2> $OUT/$tag/pmc_$ctr.err || return 1
  done
  python3 tools/pmc_traffic.py $OUT/$tag $OUT/$tag/pmc_traffic.json $kern > $OUT/$tag/pmc.log 2>&1 || return 1
  cp $OUT/$tag/pmc_traffic.json profiles/r06/$name || return 1
  cp $OUT/$tag/pmc_traffic.json $OUT/$name || return 1
}
pmc pmc_head k_service pmc_traffic.json --steps 2 --warmup 1 || exit 1
pmc pmc_horizon k_service pmc_traffic_horizon1000.json --steps 1 --warmup 1 --horizon 1000 || exit 1
pmc pmc_reference k_service pmc_traffic_reference.json --steps 1 --warmup 1 --schedule reference || exit 1
pmc pmc_init k_service pmc_traffic_init.json --steps 1 --warmup 1 --dist init || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --horizon 1000 > $OUT/bench_horizon.json 2> $OUT/bench_horizon.err || exit 1
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --schedule reference > $OUT/bench_reference.json 2> $OUT/bench_reference.err || exit 1
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --dist init > $OUT/bench_init.json 2> $OUT/bench_init.err || exit 1
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so >> $OUT/lib_sha.txt  # unchanged: nothing rebuilt it
echo done > $OUT/ok
