set -o pipefail
mkdir -p gpurun_out/w10
PG_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --config wide --pop 2048 --no-cpu-baseline > gpurun_out/w10/wide_n2.json 2> gpurun_out/w10/wide_n2.err || exit 1
timeout -k 10 300 python bench.py --config wide --pop 2048 --no-cpu-baseline > gpurun_out/w10/wide_n1.json 2> gpurun_out/w10/wide_n1.err || exit 1
