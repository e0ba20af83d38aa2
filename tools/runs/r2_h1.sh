# round 2, session 4, call h1: the committed build once more -- GPU suite and smoke
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_h1; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit 1
echo done > $OUT/ok
