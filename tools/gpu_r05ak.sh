#!/bin/bash
# C4 4K/512 whole frame: group order settings (NART_RQ_TOPF, NART_PROBE_SUB, NART_RQ_ORDER).
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r05ak_c4_order.log
: > $L
run() { echo "== $*" >> $L; env "$@" timeout -k 10 120 python -u tools/shard_perf.py --config c4 --ns 1 --reps 1 >> $L 2>&1; }
run X=1 && run NART_RQ_TOPF=5 && run NART_RQ_TOPF=20 && run NART_PROBE_SUB=16 && run NART_RQ_ORDER=0 && run NART_RQ_ORDER=1 && run X=1
