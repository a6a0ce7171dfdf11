#!/bin/bash
# Light records at uniform indices through the constant address space (scalar loads).  Parity, then
# per-kernel times under rocprofv3: C3 1080p/256, C5 1080p/256, new vs base, twice.
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r05z2_pytest.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for v in new base new base; do
  if [ $v = base ]; then export NART_HIP_LIB=$R/abbuild/nosc/libnart_hip.so; else unset NART_HIP_LIB; fi
  for sc in glass c5 c4; do
    n=${v}_${sc}_$RANDOM
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r05z2/$n -o run -- python3 $R/tools/quick_perf.py --scene $sc -w 1920 -H 1080 -s $([ $sc = c4 ] && echo 32 || echo 256) --reps 2 > $R/gpurun_out/prof_r05z2_$n.log 2>&1 || exit 1
  done
done
