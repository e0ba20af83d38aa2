# round 6: cycles per stage of serve_inline (PG_SERVE_STAGES) on the
# evolved U[0,1) population and the N(0,3) one; the product's bench lines.
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_c8}
OUT=gpurun_out/$TAG; mkdir -p $OUT
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so ab/*.so > $OUT/lib_sha.txt
PONG_GA_LIB=ab/stages.so timeout -k 10 300 python3 -u tools/init_probe.py stages 3 uniform > $OUT/stages_init.log 2>&1 || exit 1
PONG_GA_LIB=ab/stages.so timeout -k 10 300 python3 -u tools/init_probe.py stages 3 normal > $OUT/stages_normal.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --dist init --steps 5 --warmup 2 --no-cpu-baseline > $OUT/init_product_1.json 2>> $OUT/err.log || exit 1
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/head_product_1.json 2>> $OUT/err.log || exit 1
echo done > $OUT/ok
