#!/bin/bash
# k_primary: triangle records in pairs in the packet traversal.  Parity (primary / frames), then
# C3 and C4 A/B with rocprofv3 kernel times.
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r05u_packet_pairs_ab.log
: > $L
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_frames.py -k "primary or packet or c3 or c4" > gpurun_out/r05u_pytest.log 2>&1 || exit 1
for v in new base new base; do
  if [ $v = base ]; then export NART_HIP_LIB=abbuild/nopk/libnart_hip.so; else unset NART_HIP_LIB; fi
  echo "== $v" >> $L
  timeout -k 10 120 python -u tools/quick_perf.py -w 1920 -H 1080 -s 256 --reps 2 >> $L 2>&1 || exit 1
  timeout -k 10 120 python -u tools/quick_perf.py --scene c4 -w 1920 -H 1080 -s 32 --reps 2 >> $L 2>&1 || exit 1
done
unset NART_HIP_LIB
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r05u -o run -- python3 $GRAFT_REPO_ROOT/tools/quick_perf.py -w 1920 -H 1080 -s 256 --reps 2 > $GRAFT_REPO_ROOT/gpurun_out/r05u_prof.log 2>&1
