# round 3, call i6: serve table in LDS (Pong::serve_entry per game slot) --
# the whole -m gpu suite, same-box A/B against the i5 library (sweep + bench),
# SQ counters of the new library
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_i6}; mkdir -p $OUT
B=variants/base_i5.so; N=neuro-genetic-pong-self-play_amd/libpong_ga.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 900 python -u tools/sweep.py --libs $B,$N,$B,$N,$B,$N --lanes 8 --reps 5 --kernel split > $OUT/sweep.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
PONG_GA_LIB=$B timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_base.json 2> $OUT/bench_base.err || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench2.json 2> $OUT/bench2.err || exit 1
bash tools/pmc_resident.sh ${RUN:-r3_i6}/sq 8 || exit 1
python3 tools/pmc_summary.py $OUT/sq > $OUT/sq_summary.txt 2>&1 || exit 1
echo done > $OUT/ok
