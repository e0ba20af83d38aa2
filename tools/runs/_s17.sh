set -o pipefail
mkdir -p gpurun_out/s17
L=neuro-genetic-pong-self-play_amd/libpong_ga.so
timeout -k 10 600 python -u tools/sweep.py --libs $L,variants/lib_ilb1.so,variants/lib_ilb4.so,variants/lib_slp.so,$L --lanes 8 --reps 5 > gpurun_out/s17/sweep.log 2>&1 || exit 1
