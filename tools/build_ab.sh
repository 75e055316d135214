#!/bin/bash
# A/B build of the product library with extra compile flags:
#   tools/build_ab.sh NAME "-DFLAG=1 ..."  →  libhpc_amd/_abx/NAME/liblhpc.so (+ liblhpc_probe.so)
# Loaded on the box by `tools/gpu.sh OUT "benv X LHPC_LIB_PATH=libhpc_amd/_abx/NAME/liblhpc.so ..."`.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
make -C "$R/libhpc_amd/csrc" -j8 BUILD="../_build_abx_$1" OUT="../_abx/$1" EXTRA_HIPFLAGS="$2" EXTRA_CXXFLAGS="$2" \
  "../_abx/$1/liblhpc.so" "../_abx/$1/liblhpc_probe.so" > "/tmp/build_ab_$1.log" 2>&1 || { tail -20 "/tmp/build_ab_$1.log"; exit 1; }
echo "built libhpc_amd/_abx/$1 ($2)"
