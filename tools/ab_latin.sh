#!/bin/bash
# LatinSquare index-shuffle A/B on the GPU box (repo root): the GPU LatinSquare parity tests of the
# default build first, then C5 (1080p/1024) timings of each named build.
#   tools/ab_latin.sh TAG name...   (name "default" = nart_amd/lib, others abbuild/<name>/)
TAG=${1:?tag}; shift
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "latin" -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_parity.log 2>&1 || { echo parity failed; tail -20 gpurun_out/${TAG}_parity.log; exit 1; }
tail -1 gpurun_out/${TAG}_parity.log
for v in "$@"; do
  if [ $v = default ]; then unset NART_HIP_LIB; else export NART_HIP_LIB=abbuild/$v/libnart_hip.so; fi
  timeout -k 10 200 python -u tools/quick_perf.py --scene c5 -s 1024 --reps 3 >> gpurun_out/${TAG}_$v.log 2>&1 \
      || { echo "$v failed"; tail -5 gpurun_out/${TAG}_$v.log; exit 1; }
  grep '^{' gpurun_out/${TAG}_$v.log | tail -3 | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$v', 'latin_ms %.2f kernel_ms %.2f splat_ms %.2f' % (d['latin_ms'], d['kernel_ms'], d['splat_ms']))"
done
