# round 5, call b1: the round-4 library as shipped (the round's starting point):
# the whole -m gpu suite, the driver's bench command, a rocprof kernel trace of
# it, the FETCH_SIZE / WRITE_SIZE PMC passes of the headline, and the SQ
# counters of k_service (two passes of one launch on the bench workload)
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r5_b1}
OUT=gpurun_out/$TAG; mkdir -p $OUT; ROOT=$(pwd)
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so > $OUT/lib_sha.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof -o kt -- python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
mkdir -p $OUT/pmc_head
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_head/pmc_$ctr -o pmc -- python3 $ROOT/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $OUT/pmc_head/pmc_$ctr.json 2> $OUT/pmc_head/pmc_$ctr.err || exit 1
done
python3 tools/pmc_traffic.py $OUT/pmc_head $OUT/pmc_head/pmc_traffic.json k_service > $OUT/pmc_head/pmc.out 2>&1 || exit 1
bash tools/pmc_sq.sh $TAG/sq 8 || exit 1
python3 tools/pmc_summary.py $OUT/sq > $OUT/sq_summary.txt 2>&1 || exit 1
echo done > $OUT/ok
