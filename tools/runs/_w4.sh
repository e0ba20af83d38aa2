set -o pipefail
mkdir -p gpurun_out/w4
export TMPDIR=/tmp
for sh in 6,512,512,3 6,511,512,3 6,447,512,3; do
  PG_SHAPE=$sh PONG_GA_LIB=$PWD/variants/lib_stamps.so timeout -k 10 300 python -u tools/wide_probe.py 4096 >> gpurun_out/w4/probe.log 2>&1 || exit 1
  echo "^^ $sh" >> gpurun_out/w4/probe.log
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $PWD/gpurun_out/w4/pmc -o pmc -- python3 tools/wide_probe.py 2048 > gpurun_out/w4/pmc.log 2>&1 || exit 2
