#!/bin/bash
# Build an A/B variant of libmtgpu.so with extra flags for the LDS engine (mt_apply.hip) only:
#   tools/build_variant_apply.sh NAME "-DMT_LOC_WPE=3"   ->  ablib/libmtgpu_NAME.so
# The other objects are the in-tree build's (python fluidframework_amd/build.py first).
set -e
cd "$(dirname "$0")/.."
NAME=$1; FLAGS=$2
mkdir -p ablib
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-result \
  -Wno-unused-value $FLAGS -c fluidframework_amd/csrc/mt_apply.hip -o ablib/${NAME}_apply.o
B=fluidframework_amd/build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ablib/libmtgpu_${NAME}.so ablib/${NAME}_apply.o $B/mt_apply_reg.hip.o \
  $B/mt_service.hip.o $B/mt_deli.hip.o $B/mt_engine.cpp.o $B/mt_comm.cpp.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo ablib/libmtgpu_${NAME}.so
