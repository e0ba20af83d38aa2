set -o pipefail
mkdir -p gpurun_out/s1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_evolve.py tests/test_gpu_dist.py tests/test_gpu_replay.py > gpurun_out/s1/tests.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/ga_profile.py 524288 3 > gpurun_out/s1/profile_524k.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/ga_profile.py 65536 4 > gpurun_out/s1/profile_65k.log 2>&1 || exit 1
