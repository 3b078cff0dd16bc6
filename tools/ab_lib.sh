#!/bin/bash
# A/B variant of libpnol_amd.so: the kernels rebuilt with extra defines into _ab/NAME/, the host
# objects linked from the in-tree build.  Load it with PNOL_AMD_LIB=_ab/NAME/libpnol_amd.so.
#   tools/ab_lib.sh NAME -DPNOL_CHOL_MP=0 ...
set -eu
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/parallelnonlinearoptimizationlibrary_amd
OUT=$ROOT/_ab/$NAME
mkdir -p "$OUT"
make -s -C "$PKG/csrc" -j8
FLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -I$ROOT/include -I$PKG/csrc --offload-arch=gfx950 -munsafe-fp-atomics $*"
objs=()
for f in "$PKG"/csrc/kernels/*.hip; do
  o=$OUT/k_$(basename "$f" .hip).o
  /opt/rocm/bin/hipcc $FLAGS -c "$f" -o "$o" &
  objs+=("$o")
done
wait
host=$(ls "$PKG"/_build/*.o | grep -v '/k_')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -o "$OUT/libpnol_amd.so" "${objs[@]}" $host -shared -L/opt/rocm/lib -lamdhip64 -lrccl -Wl,-rpath,/opt/rocm/lib
echo "$OUT/libpnol_amd.so"
