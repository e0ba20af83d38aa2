# round 4, call a2: k_wide spill-free build (game records and counters in
# LDS, loop-opaque thread index) -- the wide parity tests, a same-box A/B
# against the round-3 k_wide (variants/lib_wide_r3.so), the FETCH/WRITE PMC
# passes of bench --config wide, then the wide bench line reading them, and
# its rocprof kernel trace
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r4_a2}; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_wide.log 2>&1 || exit 1
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
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof_wide -o kt -- python3 $ROOT/bench.py --config wide --no-cpu-baseline > $OUT/prof_wide.json 2> $OUT/prof_wide.err || exit 1
echo done > $OUT/ok
