#!/bin/bash
# Sensitivity of k_render_rq to the number of BVH nodes staged in LDS (C3 scene, 1080p / 64 spp).
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r05q_lds_nodes.log
: > $L
for n in default 0 128 256 512 640; do
  if [ $n = default ]; then unset NART_LDS_NODES; else export NART_LDS_NODES=$n; fi
  echo "== nodes $n" >> $L
  timeout -k 10 120 python -u tools/quick_perf.py -w 1920 -H 1080 -s 64 --reps 2 >> $L 2>&1 || exit 1
done
unset NART_LDS_NODES
echo "== counters" >> $L
timeout -k 10 120 python -u tools/quick_perf.py -w 1920 -H 1080 -s 16 --reps 1 --counters >> $L 2>&1
