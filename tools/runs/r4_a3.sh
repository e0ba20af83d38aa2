# round 4, call a3: the game ring in k_service (the service wave stages claimed
# games' schedule entries and lane records in LDS) + the spill-free k_wide --
# the whole -m gpu suite, a same-box A/B of the split kernel against the
# round's previous k_service (variants/lib_svc_base.so), the headline bench,
# then the wide A/B against the round-3 k_wide (variants/lib_wide_r3.so), the
# FETCH/WRITE PMC passes of bench --config wide and the wide bench line
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r4_a3}; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for i in 1 2; do
  for L in neuro-genetic-pong-self-play_amd/libpong_ga.so variants/lib_svc_base.so; do
    timeout -k 10 300 python -u tools/sweep.py --libs $L --lanes 0 --reps 3 >> $OUT/sweep_ring_ab.log 2>&1 || exit 1
  done
done
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
for i in 1 2; do
  for L in neuro-genetic-pong-self-play_amd/libpong_ga.so variants/lib_wide_r3.so; do
    timeout -k 10 300 python -u tools/sweep.py --libs $L --lanes 0 --reps 2 --kernel wide --shape 6,512,512,3 --pop 16384 --dtype f32 >> $OUT/sweep_wide_ab.log 2>&1 || exit 1
  done
done
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_$ctr -o pmc -- python3 $ROOT/bench.py --config wide --no-cpu-baseline > $OUT/pmc_$ctr.json 2> $OUT/pmc_$ctr.err || exit 1
done
python3 tools/pmc_traffic.py $OUT $OUT/pmc_traffic_wide.json k_wide > $OUT/pmc.log 2>&1 || exit 1
mkdir -p profiles/r04 && cp $OUT/pmc_traffic_wide.json profiles/r04/pmc_traffic_wide.json
timeout -k 10 600 python3 -u bench.py --config wide --gpus 1 --steps 2 --warmup 1 > $OUT/bench_wide.json 2> $OUT/bench_wide.err || exit 1
echo done > $OUT/ok
