#!/bin/bash
# round 5: k_splat_rows prefetch depth (4 default / 8 / 16) on small shards; rows vs skew on whole
# frames; then a PC-sampling attempt on the path kernel (line-table build), last
step() { tools/gpu_step.sh "$@" || exit 1; }
for v in rpf8 rpf16; do
  NART_HIP_LIB=abbuild/$v/libnart_hip.so step r05f_c5_$v 300 python -u tools/shard_perf.py --config c5 --ns 4 8 --reps 2 --rank 0
  NART_HIP_LIB=abbuild/$v/libnart_hip.so step r05f_c3_$v 300 python -u tools/shard_perf.py --config c3 --ns 8 --reps 2 --rank 0
done
step r05f_c5_pf4 300 python -u tools/shard_perf.py --config c5 --ns 4 8 --reps 2 --rank 0
NART_SPLAT_MODE=5 step r05f_c5_full_rows 300 python -u tools/shard_perf.py --config c5 --ns 1 --reps 2
NART_SPLAT_MODE=4 step r05f_c5_full_skew 300 python -u tools/shard_perf.py --config c5 --ns 1 --reps 2
NART_SPLAT_MODE=5 step r05f_c3_full_rows 300 python -u tools/shard_perf.py --config c3 --ns 1 --reps 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
NART_HIP_LIB=abbuild/pcs/libnart_hip.so timeout -s KILL 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 50 --output-format csv -d gpurun_out/pcs -o pcs -- python3 tools/quick_perf.py -s 32 --reps 1 > gpurun_out/r05f_pcs.log 2>&1
echo "pcs rc=$?"
ls -R gpurun_out/pcs | head -20
echo all-done
