set -o pipefail
for v in lk1 lk4 lnoswap lnogather; do
  NART_HIP_LIB=abbuild/$v/libnart_hip.so tools/gpu_step.sh ab_$v 200 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline || exit 1
done
NART_BATCH_BYTES=100000000000 tools/gpu_step.sh bb_c5_s3 300 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline || exit 1
NART_BATCH_BYTES=100000000000 NART_SPLAT_MODE=5 tools/gpu_step.sh bb_c5_s5 300 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline || exit 1
NART_BATCH_BYTES=130000000000 tools/gpu_step.sh bb_c4 600 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline || exit 1
