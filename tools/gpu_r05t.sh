#!/bin/bash
# Triangle record group size K (0 = one at a time, 2, 3, 4) and BVH leaf size, C3 1080p/256.
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r05t_tri_group_ab.log
: > $L
run() { echo "== $1 $2" >> $L; if [ $1 = k2 ]; then unset NART_HIP_LIB; else export NART_HIP_LIB=abbuild/$1/libnart_hip.so; fi
        env $2 timeout -k 10 120 python -u tools/quick_perf.py -w 1920 -H 1080 -s 256 --reps 2 >> $L 2>&1; }
for r in 1 2; do
  run k2 "X=1" && run tri3 "X=1" && run tri4 "X=1" && run notpf "X=1" || exit 1
done
run tri4 "NART_BVH_LEAF=8" && run tri4 "NART_BVH_LEAF=6" && run tri4 "NART_BVH_LEAF_SAH=16" && run k2 "NART_BVH_LEAF=6" && run notpf "NART_BVH_LEAF=6"
