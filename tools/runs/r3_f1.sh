# round 3, call f1: k_wide pinned by itself (pg_wide_decide on the 1 500
# near-ties), config 5 at pop 4 096 with an oracle re-check, the counters
# this rocprofv3 offers (MALL?), and a same-box A/B of k_wide before/after
# the probe entry at pop 4 096
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_f1}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_hard_cases.py tests/test_gpu_wide.py -x -v -s --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 600 python -u tools/sweep.py --libs variants/lib_widehead.so,neuro-genetic-pong-self-play_amd/libpong_ga.so,variants/lib_widehead.so,neuro-genetic-pong-self-play_amd/libpong_ga.so --lanes 0 --reps 2 --kernel wide --shape 6,512,512,3 --pop 4096 --dtype f32 > $OUT/sweep_wide.log 2>&1 || exit 1
echo done > $OUT/ok
