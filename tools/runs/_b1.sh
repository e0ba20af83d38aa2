set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/b1
timeout -k 10 600 python -u bench.py > gpurun_out/b1/bench.json 2> gpurun_out/b1/bench.err || exit 1
PG_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 > gpurun_out/b1/bench_n2_gloo.json 2> gpurun_out/b1/bench_n2.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $(pwd)/gpurun_out/b1/prof -o bench -- python3 bench.py --no-cpu-baseline > gpurun_out/b1/bench_prof.json 2> gpurun_out/b1/prof.err || exit 1
