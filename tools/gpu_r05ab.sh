#!/bin/bash
# k_latin_emit with an XCD-aware block order.  Latin parity tests, then C5 1080p/1024 and C3
# 1080p/256 per-kernel times (rocprofv3) and one FETCH_SIZE pass each, new vs base.
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "latin" > gpurun_out/r05ab_pytest.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for v in new base new base; do
  if [ $v = base ]; then export NART_HIP_LIB=$R/abbuild/noxcd/libnart_hip.so; else unset NART_HIP_LIB; fi
  for sc in c5 glass; do
    n=${v}_${sc}_$RANDOM
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r05ab/$n -o run -- python3 $R/tools/quick_perf.py --scene $sc -w 1920 -H 1080 -s $([ $sc = c5 ] && echo 1024 || echo 256) --reps 2 > $R/gpurun_out/prof_r05ab_$n.log 2>&1 || exit 1
  done
done
for v in new base; do
  if [ $v = base ]; then export NART_HIP_LIB=$R/abbuild/noxcd/libnart_hip.so; else unset NART_HIP_LIB; fi
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof_r05ab/fetch_$v -o run -- python3 $R/tools/quick_perf.py --scene c5 -w 1920 -H 1080 -s 1024 --reps 1 > $R/gpurun_out/prof_r05ab_fetch_$v.log 2>&1 || exit 1
done
