# round 3, call a1: this round's baseline on the committed build -- the
# driver's bench command, then a kernel + memory-copy trace of a short bench
# run for the per-generation device-idle gaps
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_a1}; mkdir -p $OUT
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $(pwd)/$OUT/prof -o kt -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
echo done > $OUT/ok
