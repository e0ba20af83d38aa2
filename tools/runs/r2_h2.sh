# round 2, session 4, call h2: the bench's N > 1 path rehearsed on one GPU
# (two gloo ranks sharing the device; a code-path check, not a scaling number)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_h2; mkdir -p $OUT
PG_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 > $OUT/bench_n2_gloo.json 2> $OUT/bench_n2_gloo.err || exit 1
echo done > $OUT/ok
