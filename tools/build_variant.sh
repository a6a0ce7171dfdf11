#!/bin/bash
# Build a compile-time variant of the render library on the CPU (no GPU needed), for A/B timing
# on the GPU box without spending GPU time on compiles:
#   tools/build_variant.sh NAME "-DFLAG=1 ..."   ->  abbuild/NAME/libnart_hip.so
# Run it with NART_HIP_LIB=abbuild/NAME/libnart_hip.so (nart_amd/api.py).
NAME=$1; FLAGS=$2
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/abbuild/$NAME"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -std=c++17 -O3 -fPIC \
  -ffp-contract=off -fno-fast-math -w $FLAGS -shared -o "$R/abbuild/$NAME/libnart_hip.so" \
  "$R/nart_amd/csrc/render.hip" "$R/nart_amd/csrc/host/bvh_build.cpp" -L"$R/nart_amd/lib" -lnart_scene \
  -Wl,-rpath,'$ORIGIN/../../nart_amd/lib'
