#!/bin/bash
# Build a libpong_ga.so variant with extra defines for pong_ga.hip (k_service & co.),
# linking the main build's other objects: variants/lib_NAME.so.
# usage: tools/build_variant.sh NAME [-DFLAG=VALUE ...]   (run the main build first)
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/neuro-genetic-pong-self-play_amd/csrc
mkdir -p $ROOT/variants
# the main build's machine scheduler for pong_ga.hip (pong_amd/build.py SOURCE_FLAGS); PG_SCHED overrides
SCHED=${PG_SCHED:-iterative-ilp}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -Wall \
  -Wno-unused-function -I $ROOT/include -mllvm -amdgpu-sched-strategy=$SCHED "$@" -c -o /tmp/pg_variant_$NAME.o \
  $C/pong_ga.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $ROOT/variants/lib_$NAME.so /tmp/pg_variant_$NAME.o \
  $C/pg_wide.o $C/pg_pixels.o
echo $ROOT/variants/lib_$NAME.so
