# round 2, session 4, call g1: GA step profile at P = 524 288 and 65 536 on
# the committed build (per-rank replicated work for DESIGN 7)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_g1; mkdir -p $OUT
timeout -k 10 300 python -u tools/ga_profile.py 524288 8 > $OUT/ga_profile_524k.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ga_profile.py 65536 8 > $OUT/ga_profile_65k.log 2>&1 || exit 1
echo done > $OUT/ok
