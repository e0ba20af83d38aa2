# round 6, the final library, call 2 of 2: the HBM ceiling runs; the wide PMC
# passes and its bench line (5 timed steps); a rocprof kernel trace with stats of the driver's
# bench command; the SQ counters of k_service; the N = 8 scale model.
# Afterwards gpurun_out/<tag>/* is copied into profiles/r06/ (*_final.*).
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_final2}
OUT=gpurun_out/$TAG; mkdir -p $OUT; ROOT=$(pwd)
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so > $OUT/lib_sha.txt
# the box's streaming-read ceiling with k_wide's load shape (bench.py's wide
# line reads profiles/r06/hbm_ceiling.jsonl)
for cfg in "8 5 1 2" "8 5 1 4" "8 5 2 1" "8 5 2 2" "8 5 2 4" "8 5 4 1" "8 5 4 2" "8 5 4 4" "16 5 2 2" "16 5 2 4"; do
  timeout -k 10 120 tools/bin/hbm_ceiling $cfg >> $OUT/hbm_ceiling.jsonl 2>> $OUT/err.log || exit 1
done
cp $OUT/hbm_ceiling.jsonl profiles/r06/hbm_ceiling.jsonl || exit 1
mkdir -p $OUT/pmc_wide
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_wide/pmc_$ctr -o pmc -- python3 $ROOT/bench.py --no-cpu-baseline --config wide > $OUT/pmc_wide/pmc_$ctr.json 2> $OUT/pmc_wide/pmc_$ctr.err || exit 1
done
python3 tools/pmc_traffic.py $OUT/pmc_wide $OUT/pmc_traffic_wide.json k_wide > $OUT/pmc_wide/pmc.log 2>&1 || exit 1
cp $OUT/pmc_traffic_wide.json profiles/r06/ || exit 1
timeout -k 10 900 python3 -u bench.py --config wide --gpus 1 --steps 5 --warmup 1 > $OUT/bench_wide.json 2> $OUT/bench_wide.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof -o kt -- python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
bash tools/pmc_sq.sh $TAG/sq 8 || exit 1
python3 tools/pmc_summary.py $OUT/sq > $OUT/sq_summary.txt 2>&1 || exit 1
timeout -k 10 600 python3 -u tools/scale_model.py 8 4 > $OUT/scale_model.log 2>&1 || exit 1
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so >> $OUT/lib_sha.txt  # unchanged: nothing rebuilt it
echo done > $OUT/ok
