set -o pipefail
export TMPDIR=/tmp
bash tools/pmc_resident.sh pmc_svc 8 || exit 1
OUT=gpurun_out/pmc_svc
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_FLAT SQ_INSTS_VALU_CVT --kernel-trace --output-format csv -d $(pwd)/$OUT/p3 -o pmc -- python3 tools/sweep.py --one --lane=8 --reps 1 > $OUT/p3.out 2> $OUT/p3.err
echo "pass 3 exit=$?" >> $OUT/summary.txt
