#!/bin/bash
# A/B timing of compile-time variants of the render library (GPU box, repo root).
#   tools/ab.sh OUTDIR SPP "name1:-DFLAG=1 -DX" "name2:" ...
# Builds each variant into OUTDIR/<name>/libnart_hip.so and times tools/quick_perf.py on it.
OUT=$1; SPP=$2; shift 2
mkdir -p $OUT
R=$(pwd)
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  mkdir -p $OUT/$name
  timeout -k 10 300 /opt/rocm/bin/hipcc --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -std=c++17 -O3 -fPIC \
    -ffp-contract=off -fno-fast-math -w $flags -shared -o $OUT/$name/libnart_hip.so nart_amd/csrc/render.hip \
    nart_amd/csrc/host/bvh_build.cpp -L$R/nart_amd/lib -lnart_scene -Wl,-rpath,$R/nart_amd/lib || exit 1
  echo "== $name ($flags)"
  NART_HIP_LIB=$OUT/$name/libnart_hip.so timeout -k 10 300 python tools/quick_perf.py -s $SPP --reps 2 | tail -1 | \
    python -c "import json,sys; d=json.loads(sys.stdin.read()); print('kernel_ms %.2f splat_ms %.2f Msps %.1f' % (d['kernel_ms'], d['splat_ms'], d['msamples_per_s_kernel']))" || exit 1
done
