#!/bin/bash
# Experiment builds of the product library with compile-time knobs, for A/B timing on the box:
#   tests/build_variant.sh <name> -DKNOB=VALUE ...  ->  build_exp/<name>/libsiftgpu.so
# Load one with SGPU_LIB_PATH=build_exp/<name>/libsiftgpu.so (tests/probe.py, bench.py).
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/build_exp/$NAME
mkdir -p "$OUT"
PKG=$ROOT/modify-sift-gpu_amd
FP="-ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt"
CX="-O3 -std=c++17 -fPIC --offload-arch=gfx950 $FP -I$ROOT/include -I$PKG/csrc $*"
H=/opt/rocm/bin/hipcc
$H $CX -c -o "$OUT/k.o" $PKG/csrc/sift_kernels.hip &
$H $CX -c -o "$OUT/d.o" $PKG/csrc/sift_gauss_duo.hip &
$H $CX -c -o "$OUT/t.o" $PKG/csrc/sift_gauss_tile.hip &
$H $CX -c -o "$OUT/r.o" $PKG/csrc/sift_gauss_trio.hip &
$H $CX -mllvm -amdgpu-mfma-vgpr-form=1 -c -o "$OUT/m.o" $PKG/csrc/sift_match.hip &
$H $CX -x hip -c -o "$OUT/c.o" $PKG/csrc/sgpu_capi.cpp &
$H $CX -x hip -c -o "$OUT/a.o" $PKG/csrc/siftgpu_api.cpp &
wait
$H --offload-arch=gfx950 -shared -o "$OUT/libsiftgpu.so" "$OUT"/{k,d,t,r,m,c,a}.o -L/opt/rocm/lib -lrccl -ldl -Wl,-rpath,/opt/rocm/lib
rm -f "$OUT"/*.o
# the test-hook library is loaded from beside the product library (sgpu_debug_candidates)
cp "$PKG/lib/libsiftgpu_debug.so" "$OUT/"
# a kernel whose host stub was not emitted links into the .so and fails only when loaded
if nm -D --undefined-only "$OUT/libsiftgpu.so" | grep -q __device_stub; then echo "undefined kernel stubs in $OUT"; exit 1; fi
echo "built $OUT/libsiftgpu.so"
