# round 5, call b10 (diagnostic, the product unchanged): where a k_service
# wave's time goes -- the shader cycles of the in-wave f64 decisions (until the
# reloaded output layer has landed; -DPG_DECIDE_PROBE, ab/lib_decprobe.so) and
# of the game-start blocks (-DPG_START_PROBE, ab/lib_startprobe.so) against
# the waves' total, on the sweep workload with N(0, 3) and U[0, 1) genes,
# beside the product's launch time
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r5_b10}; mkdir -p $OUT
P=neuro-genetic-pong-self-play_amd/libpong_ga.so
sha256sum $P ab/*.so > $OUT/lib_sha.txt
for d in normal uniform; do
  for L in $P ab/lib_decprobe.so ab/lib_startprobe.so; do
    timeout -k 10 300 python -u tools/sweep.py --libs $L --lanes 0 --reps 3 --dist $d >> $OUT/sweep_probe.log 2>&1 || exit 1
  done
done
echo done > $OUT/ok
