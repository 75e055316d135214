#!/bin/bash
# A/B build of the product library with extra compile flags:
#   tools/build_ab.sh NAME "-DFLAG=1 ..."  →  libhpc_amd/_abx/NAME/liblhpc.so (+ liblhpc_probe.so)
# Loaded on the box by `tools/gpu.sh OUT "benv X LHPC_LIB_PATH=libhpc_amd/_abx/NAME/liblhpc.so ..."`.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
# -DLHPC_AB_BUILD: lhpc_build_flags() reports LHPC_BUILD_AB whatever the flags
make -C "$R/libhpc_amd/csrc" -j8 BUILD="../_build_abx_$1" OUT="../_abx/$1" EXTRA_HIPFLAGS="$2 -DLHPC_AB_BUILD" \
  EXTRA_CXXFLAGS="$2 -DLHPC_AB_BUILD" \
  "../_abx/$1/liblhpc.so" "../_abx/$1/liblhpc_probe.so" > "/tmp/build_ab_$1.log" 2>&1 || { tail -20 "/tmp/build_ab_$1.log"; exit 1; }
echo "built libhpc_amd/_abx/$1 ($2)"
