# round 2, session 3, call 12: the widened fixtures (sigma-3 episodes over every
# game slot with long rallies and timeouts, traced and untraced, split + staged;
# sigma-3 wide forwards) in the full GPU suite
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_b12; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
echo done > $OUT/ok
