#!/bin/bash
# Builds an A/B variant of libska_sdp_func.so into variants/<name>/ with one
# source file recompiled under extra flags; every other object comes from
# the in-tree build. Select it at run time with SKA_SDP_FUNC_LIB_DIR.
#   scripts/variant_lib.sh NAME csrc/visibility/sdp_flagger.hip [-Dflags...]
# REPLACES=csrc/... names the in-tree object the variant stands in for when
# SRC is a renamed copy (e.g. the HEAD version of a file under test).
set -e
NAME=$1; SRC=$2; shift 2
cd "$(dirname "$0")/../ska-sdp-func_amd"
OUT=../variants/$NAME
mkdir -p "$OUT"
REP=${REPLACES:-$SRC}
OBJ=build/$(dirname "${REP#csrc/}")/$(basename "$REP").o
CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -I/root/repo/include -Icsrc -Wall -Wno-unused-result"
# Per-file flags of the Makefile (MFMA results in VGPRs).
case "$REP" in
  *es_kernels.hip|*sdp_grid_wstack_wtower.hip) CXXFLAGS="$CXXFLAGS -mllvm -amdgpu-mfma-vgpr-form" ;;
esac
/opt/rocm/bin/hipcc $CXXFLAGS "$@" -x hip -c "$SRC" -o "$OUT/variant.o"
OBJS=$(find build -name '*.o' | sort | grep -v "^$OBJ\$")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -L/opt/rocm/lib -lrocfft -Wl,-rpath,/opt/rocm/lib -Wl,-soname,libska_sdp_func.so $OBJS "$OUT/variant.o" -o "$OUT/libska_sdp_func.so"
rm -f "$OUT/variant.o"
echo "built $OUT/libska_sdp_func.so"
