#!/bin/bash
# Build compile-time variants of the render library locally (no GPU needed), in parallel:
#   tools/ab_build.sh "name1:-DFLAG=1 -DX" "name2:" ...   ->  abbuild/<name>/libnart_hip.so
# then time them on the GPU box with tools/ab_run.sh SPP name1 name2 ...
R=$(cd "$(dirname "$0")/.." && pwd)
pids=()
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  mkdir -p $R/abbuild/$name
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt -std=c++17 -O3 -fPIC \
    -ffp-contract=off -fno-fast-math -w $flags -shared -o $R/abbuild/$name/libnart_hip.so $R/nart_amd/csrc/render.hip \
    $R/nart_amd/csrc/host/bvh_build.cpp -L$R/nart_amd/lib -lnart_scene -Wl,-rpath,'$ORIGIN/../../nart_amd/lib' \
    > $R/abbuild/$name/build.log 2>&1 && echo "built $name" ) || echo "FAILED $name" &
  pids+=($!)
done
wait
