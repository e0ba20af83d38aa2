#!/bin/bash
# SQ counters of the evaluation kernel for one variant.
# usage: tools/pmc_sq.sh TAG LANES [LIB]
TAG=$1; LANES=$2; LIB=$3
OUT=gpurun_out/$TAG; mkdir -p $OUT; ROOT=$(pwd); export TMPDIR=/tmp
[ -n "$LIB" ] && export PONG_GA_LIB=$ROOT/$LIB
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $ROOT/$OUT/p$i -o pmc -- python3 $ROOT/tools/sweep.py --one --lane=$LANES --reps 1 > $OUT/p$i.out 2> $OUT/p$i.err
  rc=$?; echo "pass $i exit=$rc" >> $OUT/summary.txt
  case $rc in 124|134|137|139) exit $rc;; esac
done
