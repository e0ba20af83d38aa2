# round 5, call b14: pg_decide (k_decide) runs the frame bound's tier as
# serve_inline does (stage 4), so the golden hard cases and the 300k-decision
# cascade test pin it: the whole -m gpu suite on that library, then the final
# measurement of it (tools/runs/r5_final.sh as RUN=r5_final5)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r5_b14}; mkdir -p $OUT
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so > $OUT/lib_sha.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_blas_order.py tests/test_gpu_hard_cases.py -m gpu -q -s -k "decide" --timeout 300 --timeout-method thread > $OUT/decide_stages.log 2>&1 || exit 1
RUN=r5_final5 bash tools/runs/r5_final.sh || exit 1
echo done > $OUT/ok
