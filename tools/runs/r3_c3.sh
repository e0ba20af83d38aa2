# round 3, call c3: lane records at game start (k_prep_records + load_rec) --
# a small evaluation, the parity suite, then the A/B sweep (previous build
# without records or jump, records only, records + serve jump) and the
# game-start probe of the record build
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_c3}; mkdir -p $OUT
timeout -k 10 120 python -u tools/sweep.py --one --lane=8 --reps 1 --pop 1024 --kernel split > $OUT/small.log 2>&1 || exit 1
grep -q env_steps $OUT/small.log || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hard_cases.py tests/test_gpu_generation.py tests/test_gpu_evolve.py -x -q --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/sweep.py --libs variants/lib_nojump.so,variants/lib_rec_nojump.so,neuro-genetic-pong-self-play_amd/libpong_ga.so,variants/lib_rec_probe.so,variants/lib_nojump.so,variants/lib_rec_nojump.so,neuro-genetic-pong-self-play_amd/libpong_ga.so --lanes 8 --reps 3 --kernel split > $OUT/sweep.log 2>&1 || exit 1
echo done > $OUT/ok
