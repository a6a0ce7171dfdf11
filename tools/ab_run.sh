#!/bin/bash
# Time prebuilt variants (tools/ab_build.sh) on the GPU box: tools/ab_run.sh SPP [--scene cornell] name1 name2 ...
SPP=$1; shift
SC=""
if [ "$1" == "--scene" ]; then SC="--scene $2"; shift 2; fi
for name in "$@"; do
  for rep in 1 2; do
    NART_HIP_LIB=abbuild/$name/libnart_hip.so timeout -k 10 300 python tools/quick_perf.py $SC -s $SPP --reps 2 | tail -1 | \
      python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name kernel_ms %.2f splat_ms %.2f Msps %.1f' % (d['kernel_ms'], d['splat_ms'], d['msamples_per_s_kernel']))" || exit 1
  done
done
