# round 4, the final library, call 2 of 2 (profiles/r04/pmc_traffic*.json from
# call 1 in the tree): the driver's bench command, the secondary runs
# (--horizon 1000, --schedule reference, --dist init), the wide line, the N = 8
# scale model, a rocprof kernel trace of the headline, the SQ counters of
# k_service, and the service-wave batch A/B on --dist init (product, batch 4,
# vs variants/svc_b1.so, batch 1)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r4_final2}; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --horizon 1000 > $OUT/bench_horizon.json 2> $OUT/bench_horizon.err || exit 1
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --schedule reference > $OUT/bench_reference.json 2> $OUT/bench_reference.err || exit 1
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --dist init > $OUT/bench_init.json 2> $OUT/bench_init.err || exit 1
timeout -k 10 600 python3 -u bench.py --config wide --gpus 1 --steps 2 --warmup 1 > $OUT/bench_wide.json 2> $OUT/bench_wide.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof -o kt -- python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
bash tools/pmc_sq.sh ${RUN:-r4_final2}/sq 8 || exit 1
python3 tools/pmc_summary.py $OUT/sq > $OUT/sq_summary.txt 2>&1 || exit 1
timeout -k 10 600 python3 -u tools/scale_model.py 8 4 > $OUT/scale_model.log 2>&1 || exit 1
for L in neuro-genetic-pong-self-play_amd/libpong_ga.so variants/svc_b1.so neuro-genetic-pong-self-play_amd/libpong_ga.so variants/svc_b1.so; do
  echo "$L" >> $OUT/bench_init_svc_ab.log
  PONG_GA_LIB=$ROOT/$L timeout -k 10 300 python3 -u bench.py --steps 6 --warmup 2 --dist init --no-cpu-baseline >> $OUT/bench_init_svc_ab.log 2>> $OUT/ab.err || exit 1
done
echo done > $OUT/ok
