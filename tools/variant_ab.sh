#!/bin/bash
# Prebuilt variant vs main at N=1 and N=8 C3 shards (GPU box): tools/variant_ab.sh name
V=$1
for n in 1 8; do
  for v in main $V main $V; do
    if [ $v == main ]; then L=$PWD/nart_amd/lib/libnart_hip.so; else L=$PWD/abbuild/$v/libnart_hip.so; fi
    NART_HIP_LIB=$L timeout -k 10 300 python -u tools/shard_perf.py --ns $n --reps 2 > gpurun_out/var.log 2>&1 || { tail -20 gpurun_out/var.log; exit 1; }
    echo "[N=$n $v] $(grep '^{' gpurun_out/var.log | cut -c1-140)"
  done
done
