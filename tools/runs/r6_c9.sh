# round 6: serve_inline's stages when the same request is served twice in a
# row (PG_SERVE_TWICE + PG_SERVE_STAGES): cold (first) vs warm (second) call.
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_c9}
OUT=gpurun_out/$TAG; mkdir -p $OUT
sha256sum ab/*.so > $OUT/lib_sha.txt
PONG_GA_LIB=ab/twice.so timeout -k 10 300 python3 -u tools/init_probe.py stages 3 uniform > $OUT/twice_init.log 2>&1 || exit 1
PONG_GA_LIB=ab/twice.so timeout -k 10 300 python3 -u tools/init_probe.py stages 3 normal > $OUT/twice_normal.log 2>&1 || exit 1
echo done > $OUT/ok
