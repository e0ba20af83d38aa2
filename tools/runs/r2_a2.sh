# round 2, call 2: numpy-order f64 paths -- GPU suite (incl. test_gpu_blas_order),
# harvest of the hard decisions on the bench distribution, a short bench and
# the wide bench (k_wide with the 4-partial-sum layer 2).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_a2; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/harvest_hard.py --out $OUT/hard_cases.npz > $OUT/harvest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 python -u bench.py --config wide --no-cpu-baseline > $OUT/bench_wide.json 2> $OUT/bench_wide.err || exit 1
python - > $OUT/numpy_box.txt 2>&1 <<'PY'
import numpy as np, platform
np.show_config()
print(platform.processor())
PY
echo done > $OUT/ok
