# round 4, call a4: the game ring staged by LDS-DMA (16 entries; built only
# with -DPG_RING=1: variants/lib_ring.so) -- the split kernel's parity tests
# on the product build, then on the ring build, a same-box A/B of the product
# (no ring) against the ring build and a ring-wait probe build, the headline bench,
# and the N = 8 weak-scaling model (tools/scale_model.py); the next generation's
# select/vary on a side stream beside the hall-of-fame update
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r4_a4}; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_evolve.py tests/test_gpu_generation.py -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_parity.log 2>&1 || exit 1
PONG_GA_LIB=$ROOT/variants/lib_ring.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_parity_ring.log 2>&1 || exit 1
for i in 1 2; do
  for L in neuro-genetic-pong-self-play_amd/libpong_ga.so variants/lib_ring.so variants/lib_ringprobe.so; do
    timeout -k 10 300 python -u tools/sweep.py --libs $L --lanes 0 --reps 3 >> $OUT/sweep_ring_ab.log 2>&1 || exit 1
  done
done
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 600 python3 -u tools/scale_model.py 8 4 > $OUT/scale_model.log 2>&1 || exit 1
echo done > $OUT/ok
