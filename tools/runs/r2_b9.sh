# round 2, session 3, call 9: k_staged per-network-wave phase timing
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_b9; mkdir -p $OUT
PONG_GA_LIB=$(pwd)/variants/lib_prof.so timeout -k 10 200 python -u tools/staged_probe.py > $OUT/staged_probe.json 2> $OUT/staged_probe.err || exit 1
echo done > $OUT/ok
