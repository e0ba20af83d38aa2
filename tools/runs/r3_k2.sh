# round 3, call k2: the final library of the round (eb53309), in-tree build 7e3a5e2d05215c5c -- the whole -m gpu suite, the driver's
# bench command, a rocprof kernel trace, the FETCH/WRITE PMC passes of
# k_service and k_prep_records, the SQ counters of k_service, the generation
# profiles at P = 524 288 / 65 536
# (the wide kernel is unchanged since h3)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_k2}; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof -o kt -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_$ctr -o pmc -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_$ctr.json 2> $OUT/pmc_$ctr.err || exit 1
done
python3 tools/pmc_traffic.py $OUT $OUT/pmc_traffic.json k_service > $OUT/pmc.log 2>&1 || exit 1
python3 tools/pmc_traffic.py $OUT $OUT/pmc_traffic_prep.json k_prep_records >> $OUT/pmc.log 2>&1 || exit 1
bash tools/pmc_resident.sh ${RUN:-r3_k2}/sq 8 || exit 1
python3 tools/pmc_summary.py $OUT/sq > $OUT/sq_summary.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ga_profile.py 524288 8 > $OUT/ga_profile_524k.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ga_profile.py 65536 8 > $OUT/ga_profile_65k.log 2>&1 || exit 1
echo done > $OUT/ok
