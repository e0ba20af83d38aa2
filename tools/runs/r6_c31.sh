# round 6: k_hof_rank_pack's two searches over LDS samples of the sorted
# arrays (one window of independent loads left) and k_hof_commit as one wave
# per hall position striding over the positions: the whole -m gpu suite on
# it; A/B of the driver's bench command against ab/c820.so (the library
# before), alternating, three each; a kernel trace with stats of the product.
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_c31}
OUT=gpurun_out/$TAG; mkdir -p $OUT; ROOT=$(pwd)
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so ab/*.so > $OUT/lib_sha.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for rep in 1 2 3; do
  for v in product c820; do
    if [ $v = product ]; then L=""; else L=ab/$v.so; fi
    PONG_GA_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/head_${v}_$rep.json 2>> $OUT/err.log || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof -o kt -- python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
echo done > $OUT/ok
