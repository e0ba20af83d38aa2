set -o pipefail
mkdir -p gpurun_out/w5
for v in NOCOMPUTE NOSTORE D1 D2 stamps; do
  PONG_GA_LIB=$PWD/variants/lib_$v.so timeout -k 10 300 python -u tools/wide_probe.py 4096 >> gpurun_out/w5/probe.log 2>&1 || exit 1
  echo "^^ $v" >> gpurun_out/w5/probe.log
done
