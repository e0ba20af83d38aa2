set -o pipefail
OUT=gpurun_out/p3; mkdir -p $OUT; ROOT=$(pwd); export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_$ctr -o pmc -- python3 $ROOT/bench.py --no-cpu-baseline > $OUT/pmc_$ctr.json 2> $OUT/pmc_$ctr.err || exit 1
done
python3 tools/pmc_traffic.py $OUT $OUT/pmc_traffic.json k_service > $OUT/pmc.log 2>&1 || exit 1
