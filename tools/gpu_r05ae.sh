#!/bin/bash
# BVH nodes in LDS with a 16-B pad per 4 nodes (bank spread of ds_read_b128).  Parity suite, then per-kernel
# times (rocprofv3) on C3 1080p/256 and C4 1080p/32, new vs base, twice; the 1/8 C3 shards.
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r05ae_pytest.log 2>&1 || exit 1
L=$R/gpurun_out/r05ae_shard.log
: > $L
for v in new base new base; do
  if [ $v = base ]; then export NART_HIP_LIB=$R/abbuild/nopad/libnart_hip.so; else unset NART_HIP_LIB; fi
  echo "== $v" >> $L
  timeout -k 10 300 python -u tools/shard_perf.py --config c3 --ns 8 --reps 2 >> $L 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for v in new base new base; do
  if [ $v = base ]; then export NART_HIP_LIB=$R/abbuild/nopad/libnart_hip.so; else unset NART_HIP_LIB; fi
  for sc in glass c4; do
    n=${v}_${sc}_$RANDOM
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r05ae/$n -o run -- python3 $R/tools/quick_perf.py --scene $sc -w 1920 -H 1080 -s $([ $sc = c4 ] && echo 32 || echo 256) --reps 2 > $R/gpurun_out/prof_r05ae_$n.log 2>&1 || exit 1
  done
done
