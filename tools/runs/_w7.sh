set -o pipefail
OUT=gpurun_out/w7; mkdir -p $OUT; ROOT=$(pwd); export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_$ctr -o pmc -- python3 $ROOT/bench.py --config wide --no-cpu-baseline > $OUT/pmc_$ctr.json 2> $OUT/pmc_$ctr.err || exit 1
done
python3 tools/pmc_traffic.py $OUT $OUT/pmc_traffic_wide.json k_wide > $OUT/pmc.log 2>&1 || exit 1
cp $OUT/pmc_traffic_wide.json profiles/r01/pmc_traffic_wide.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof_wide -o kt -- python3 $ROOT/bench.py --config wide --no-cpu-baseline > $OUT/prof_wide.json 2> $OUT/prof_wide.err || exit 1
timeout -k 10 300 python bench.py --config wide > $OUT/bench_wide.json 2> $OUT/bench_wide.err || exit 1
