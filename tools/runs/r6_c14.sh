# round 6: the driver's N > 1 launch of bench.py rehearsed on the one-GPU box
# with the shipped library (in-place hall, sliced hall, sharded variation):
# torch.distributed.run with 2 and 8 gloo ranks on cuda:0 (a code-path check,
# not a scaling number: the ranks share one GPU), and the RCCL path at world
# size 1 (PG_FORCE_DIST=1).
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_c14}
OUT=gpurun_out/$TAG; mkdir -p $OUT
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so > $OUT/lib_sha.txt
PG_FORCE_DIST=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_rccl_n1.json 2> $OUT/rccl_n1.err || exit 1
PG_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --steps 4 --warmup 1 --no-cpu-baseline > $OUT/bench_gloo_n2.json 2> $OUT/gloo_n2.err || exit 1
PG_DIST_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_gloo_n8.json 2> $OUT/gloo_n8.err || exit 1
echo done > $OUT/ok
