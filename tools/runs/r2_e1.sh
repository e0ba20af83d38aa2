# round 2, session 4, call e1: effective shader clock during k_service and
# k_wide (GRBM_GUI_ACTIVE cycles over the dispatch time)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_e1; mkdir -p $OUT
ROOT=$(pwd)
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $ROOT/$OUT/clk_svc -o pmc -- python3 tools/sweep.py --one --lane=8 --reps 1 > $OUT/clk_svc.out 2> $OUT/clk_svc.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $ROOT/$OUT/clk_wide -o pmc -- python3 tools/sweep.py --one --lane=0 --reps 1 --kernel wide --shape 6,512,512,3 --dtype f32 --pop 2048 > $OUT/clk_wide.out 2> $OUT/clk_wide.err || exit 1
echo done > $OUT/ok
