# round 3, call a2: where k_service's cycles go -- PC sampling over one
# bench-workload evaluation (PCS_METHOD stochastic: with stall reasons;
# host_trap: PCs only)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_a2}; mkdir -p $OUT
M=${PCS_METHOD:-stochastic}
if [ "$M" = stochastic ]; then U="--pc-sampling-unit cycles --pc-sampling-interval 65536"; else U="--pc-sampling-unit time --pc-sampling-interval 100"; fi
timeout -k 10 120 python3 -u tools/sweep.py --one --lane=8 --reps 1 --pop 65536 --kernel split > $OUT/plain.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $M $U --output-format csv -d $(pwd)/$OUT/pcs -o pcs -- python3 -u tools/sweep.py --one --lane=8 --reps 1 --pop 65536 --kernel split > $OUT/pcs.log 2>&1 || exit 1
echo done > $OUT/ok
