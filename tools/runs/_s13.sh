set -o pipefail
mkdir -p gpurun_out/s13
L=neuro-genetic-pong-self-play_amd/libpong_ga.so
timeout -k 10 600 python -u tools/sweep.py --libs $L,variants/lib_maxilp.so,variants/lib_itminreg.so,variants/lib_trackers.so,variants/lib_o2.so,$L --lanes 8 --reps 5 > gpurun_out/s13/sweep.log 2>&1 || exit 1
