# round 3, call k4: bench.py's N > 1 path on the final library, rehearsed on
# one GPU (two gloo ranks on cuda:0; a code-path check, not a scaling number),
# and the driver's N = 1 command once more
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_k4}; mkdir -p $OUT
PG_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_n2_gloo.json 2> $OUT/bench_n2_gloo.err || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
echo done > $OUT/ok
