#!/bin/bash
# Build a libpong_ga.so variant with extra defines for one translation unit
# (default pong_ga.hip: k_service & co.; PG_TU=pg_wide.hip for k_wide),
# linking the main build's other objects: ab/lib_NAME.so.
# usage: [PG_TU=pg_wide.hip] tools/build_variant.sh NAME [-DFLAG=VALUE ...]   (run the main build first)
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/neuro-genetic-pong-self-play_amd/csrc
TU=${PG_TU:-pong_ga.hip}
mkdir -p $ROOT/ab
# the main build's machine scheduler for pong_ga.hip (pong_amd/build.py SOURCE_FLAGS); PG_SCHED overrides
if [ "$TU" = "pong_ga.hip" ]; then SCHED=${PG_SCHED:-iterative-ilp}; else SCHED=${PG_SCHED:-}; fi
SFLAG=""; [ -n "$SCHED" ] && SFLAG="-mllvm -amdgpu-sched-strategy=$SCHED"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -Wall \
  -Wno-unused-function -I $ROOT/include $SFLAG "$@" -c -o /tmp/pg_variant_$NAME.o $C/$TU
OBJS="/tmp/pg_variant_$NAME.o"
for o in $C/*.o; do
  [ "$(basename $o .o).hip" = "$TU" ] || OBJS="$OBJS $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $ROOT/ab/lib_$NAME.so $OBJS
echo $ROOT/ab/lib_$NAME.so
