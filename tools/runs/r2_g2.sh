# round 2, session 4, call g2: the longest-first order test; hall-of-fame
# prepare probe at config-4 sizes
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_g2; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_evolve.py -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/diag/hof_prepare_probe.py 15000 > $OUT/probe_15k.json 2> $OUT/probe.err || exit 1
timeout -k 10 120 python -u tools/diag/hof_prepare_probe.py 150000 > $OUT/probe_150k.json 2>> $OUT/probe.err || exit 1
echo done > $OUT/ok
