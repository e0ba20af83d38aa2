set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $(pwd)/gpurun_out/s3/prof -o ga -- python3 tools/ga_profile.py 524288 3 > gpurun_out/s3/ga.log 2>&1 || exit 1
