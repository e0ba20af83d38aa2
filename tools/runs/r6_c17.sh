# round 6: unsharded, the next generation's side-stream work enqueued behind
# the merge before the host waits on it (evolve.DeviceGA.presubmit): the whole
# -m gpu suite on it; A/B of the driver's bench command against
# PG_NO_PRESUBMIT=1, alternating, three each; the host-side profile.
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_c17}
OUT=gpurun_out/$TAG; mkdir -p $OUT
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so > $OUT/lib_sha.txt
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for rep in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/head_product_$rep.json 2>> $OUT/err.log || exit 1
  PG_NO_PRESUBMIT=1 timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/head_nopre_$rep.json 2>> $OUT/err.log || exit 1
done
timeout -k 10 300 python3 -u tools/host_profile.py 20 > $OUT/host_profile.txt 2>> $OUT/err.log || exit 1
echo done > $OUT/ok
