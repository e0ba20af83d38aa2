# round 2, session 3, call 11: DeviceGA per-phase profile at the N=8 population
# (524 288, replicated per rank) and at 65 536 -- the hall-of-fame share over generations
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_b11; mkdir -p $OUT
timeout -k 10 300 python -u tools/ga_profile.py 524288 8 > $OUT/ga_profile_524k.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ga_profile.py 65536 8 > $OUT/ga_profile_65k.log 2>&1 || exit 1
echo done > $OUT/ok
