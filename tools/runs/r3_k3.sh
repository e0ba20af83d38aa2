# round 3, call k3: BASELINE config 5 (the wide [6,512,512,3] kernel) on the
# final library (Pong::step's rare blocks now behind one test there too):
# the bench line and the f32 / f64 genome-storage sweep
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_k3}; mkdir -p $OUT
timeout -k 10 600 python3 -u bench.py --config wide --gpus 1 --steps 2 --warmup 1 > $OUT/bench_wide.json 2> $OUT/bench_wide.err || exit 1
timeout -k 10 600 python -u tools/sweep.py --libs neuro-genetic-pong-self-play_amd/libpong_ga.so --lanes 0 --reps 2 --kernel wide --shape 6,512,512,3 --pop 16384 --dtype f32 > $OUT/wide_f32.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/sweep.py --libs neuro-genetic-pong-self-play_amd/libpong_ga.so --lanes 0 --reps 2 --kernel wide --shape 6,512,512,3 --pop 16384 --dtype f64 > $OUT/wide_f64.log 2>&1 || exit 1
echo done > $OUT/ok
