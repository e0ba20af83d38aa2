# round 3, call g8: the service wave polls one posted-requests word (the slot
# scan only when it moved) -- parity on the variant, A/B, SQ counters
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_g8}; mkdir -p $OUT
B=neuro-genetic-pong-self-play_amd/libpong_ga.so
PONG_GA_LIB=variants/lib_poll.so timeout -k 10 120 python -u tools/sweep.py --one --lane=8 --reps 1 --pop 1024 --kernel split > $OUT/small.log 2>&1 || exit 1
grep -q env_steps $OUT/small.log || exit 1
PONG_GA_LIB=variants/lib_poll.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hard_cases.py tests/test_gpu_evolve.py tests/test_gpu_generation.py tests/test_gpu_dropin.py -x -q --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1 || exit 1
timeout -k 10 900 python -u tools/sweep.py --libs $B,variants/lib_poll.so,$B,variants/lib_poll.so,$B,variants/lib_poll.so --lanes 8 --reps 5 --kernel split > $OUT/sweep.log 2>&1 || exit 1
bash tools/pmc_resident.sh ${RUN:-r3_g8}/sq 8 variants/lib_poll.so || exit 1
python3 tools/pmc_summary.py $OUT/sq > $OUT/sq_summary.txt 2>&1 || exit 1
echo done > $OUT/ok
