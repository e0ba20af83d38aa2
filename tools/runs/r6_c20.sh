# round 6: locality of the requests that reach serve_inline (PG_INLINE_LOG
# build with each request's wave and network): how often a wave's request
# repeats a network among its last K -- what a per-wave LDS cache of the f64
# stage's genome values would hit -- on --dist init and on N(0, 3).
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_c20}
OUT=gpurun_out/$TAG; mkdir -p $OUT
sha256sum ab/log.so > $OUT/lib_sha.txt
PONG_GA_LIB=ab/log.so timeout -k 10 300 python3 -u tools/init_probe.py $OUT/init.npz 3 uniform > $OUT/init_probe.log 2>&1 || exit 1
PONG_GA_LIB=ab/log.so timeout -k 10 300 python3 -u tools/init_probe.py $OUT/normal.npz 3 normal > $OUT/normal_probe.log 2>&1 || exit 1
echo done > $OUT/ok
