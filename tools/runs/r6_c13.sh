# round 6: the hall of fame kept in place (ABI 12: pg_hof_update_packed's
# slots, pg_hof_commit's dst_slot): the whole -m gpu suite on it; the driver's
# bench command; the N = 8 scale model with the in-place commit, the packed
# scan and the P-row preparation that reconciles the one-GPU wall at P.
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_c13}
OUT=gpurun_out/$TAG; mkdir -p $OUT
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so > $OUT/lib_sha.txt
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 600 python3 -u tools/scale_model.py 8 4 > $OUT/scale_model.log 2>&1 || exit 1
echo done > $OUT/ok
