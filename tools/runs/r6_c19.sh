# round 6: bench.py's N = 2 launch (2 gloo ranks sharing the one GPU) with the
# sharded presubmit on and off, alternating, three each (is the c18 gap real?),
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_c19}
OUT=gpurun_out/$TAG; mkdir -p $OUT
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so > $OUT/lib_sha.txt
for rep in 1 2 3; do
for v in on off; do
  if [ $v = off ]; then X=1; else X=0; fi
  PG_NO_PRESUBMIT=$X PG_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 295$rep$X bench.py --gpus 2 --steps 8 --warmup 2 --no-cpu-baseline > $OUT/gloo_n2_${v}_$rep.out 2>> $OUT/err.log || exit 1
done
done
echo done > $OUT/ok
