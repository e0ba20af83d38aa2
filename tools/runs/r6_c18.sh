# round 6: sharded, the candidates' completion and the next generation's side
# work enqueued behind the merge before the host waits on it (the completion
# over the candidate list bounded by the device-side count; k_vary's list mode
# strides over the list): the whole -m gpu suite; the driver's bench command;
# bench.py's N > 1 launch with 2 and 8 gloo ranks on the one GPU, presubmit on
# and off (a code-path check: the ranks share the GPU).
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_c18}
OUT=gpurun_out/$TAG; mkdir -p $OUT
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so > $OUT/lib_sha.txt
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/head_product_1.json 2>> $OUT/err.log || exit 1
for v in on off; do
  if [ $v = off ]; then X=1; else X=0; fi
  PG_NO_PRESUBMIT=$X PG_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2954$X bench.py --gpus 2 --steps 4 --warmup 1 --no-cpu-baseline > $OUT/gloo_n2_$v.out 2>> $OUT/err.log || exit 1
done
PG_DIST_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29549 bench.py --gpus 8 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/gloo_n8_on.out 2>> $OUT/err.log || exit 1
echo done > $OUT/ok
