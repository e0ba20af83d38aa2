set -o pipefail
mkdir -p gpurun_out/s15
L=neuro-genetic-pong-self-play_amd/libpong_ga.so
timeout -k 10 600 python -u tools/sweep.py --libs $L,variants/lib_s_max-memory-clause.so,variants/lib_s_iterative-ilp.so,variants/lib_s_iterative-maxocc.so,$L --lanes 8 --reps 5 > gpurun_out/s15/sweep.log 2>&1 || exit 1
