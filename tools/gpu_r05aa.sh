#!/bin/bash
# Volume kernel waves per SIMD on throughput-bound launches: 4 (default) vs 5 (13 VGPRs spilled) vs 3.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in wv4 wv5 wv3 wv4 wv5 wv3; do
  if [ $v = wv4 ]; then unset NART_HIP_LIB; else export NART_HIP_LIB=$R/abbuild/$v/libnart_hip.so; fi
  n=${v}_$RANDOM
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r05aa/$n -o run -- python3 $R/tools/quick_perf.py --scene c5 -w 1920 -H 1080 -s 256 --reps 2 > $R/gpurun_out/prof_r05aa_$n.log 2>&1 || exit 1
done
