# round 6: config 5's HBM evidence and its 1->8 split: the box's streaming-read
# ceiling with k_wide's load shape (tools/hbm_ceiling.hip: 1-KB non-temporal
# wave pieces, 512-thread blocks; 8 GiB, far past the Infinity Cache); the wide
# bench line with 5 timed steps; the strong-scaling model of config 5 with
# contiguous and length-balanced shards (tools/scale_model_wide.py).
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_c12}
OUT=gpurun_out/$TAG; mkdir -p $OUT
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so > $OUT/lib_sha.txt
for cfg in "8 5 1 4" "8 5 1 2" "8 5 1 8" "8 5 2 4" "16 5 1 4"; do
  timeout -k 10 120 tools/bin/hbm_ceiling $cfg >> $OUT/hbm_ceiling.jsonl 2>> $OUT/err.log || exit 1
done
timeout -k 10 900 python3 -u bench.py --config wide --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_wide.json 2>> $OUT/err.log || exit 1
timeout -k 10 900 python3 -u tools/scale_model_wide.py 2 > $OUT/scale_model_wide.log 2>&1 || exit 1
echo done > $OUT/ok
# the replicated GA work at P = 8 x 65 536 with the packed hall-of-fame scan
timeout -k 10 600 python3 -u tools/scale_model.py 8 4 > $OUT/scale_model.log 2>&1 || exit 1
echo done2 > $OUT/ok2
