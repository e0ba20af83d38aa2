set -o pipefail
mkdir -p gpurun_out/s6
timeout -k 10 600 python -u tools/ga_profile.py 524288 4 > gpurun_out/s6/profile_524k.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ga_profile.py 65536 6 > gpurun_out/s6/profile_65k.log 2>&1 || exit 1
