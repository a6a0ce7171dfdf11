#!/bin/bash
# k_primary at 4 waves per SIMD (36 VGPRs spilled) vs the allocator's 3: per-kernel times on C3
# 1080p/256 and C4 1080p/32 (rocprofv3), twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in new base new base; do
  if [ $v = new ]; then export NART_HIP_LIB=$R/abbuild/pw4/libnart_hip.so; else unset NART_HIP_LIB; fi
  for sc in glass c4; do
    n=${v}_${sc}_$RANDOM
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r05ao/$n -o run -- python3 $R/tools/quick_perf.py --scene $sc -w 1920 -H 1080 -s $([ $sc = c4 ] && echo 32 || echo 256) --reps 2 > $R/gpurun_out/prof_r05ao_$n.log 2>&1 || exit 1
  done
done
