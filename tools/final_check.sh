#!/bin/bash
# Round-end evidence pass (GPU box, repo root): parity tests, smoke, C3 bench + rocprofv3
# profile (tools/gpu_check.sh), the other BASELINE configs' bench lines, and C3/C5 shard scaling.
#   tools/final_check.sh OUT
OUT=${1:-gpurun_out/final}
bash tools/gpu_check.sh "$OUT" || exit 1
for c in c2 c4 c5; do
  timeout -k 10 400 python bench.py --config $c --steps 1 --warmup 1 > "$OUT/bench_$c.log" 2>&1 || { tail -5 "$OUT/bench_$c.log"; exit 1; }
done
timeout -k 10 600 python tools/shard_perf.py --config c3 --ns 1 2 4 8 --reps 2 > "$OUT/shard_c3.log" 2>&1 || exit 1
timeout -k 10 600 python tools/shard_perf.py --config c5 --ns 1 2 4 8 --reps 1 > "$OUT/shard_c5.log" 2>&1 || exit 1
tail -n 4 "$OUT/shard_c3.log" "$OUT/shard_c5.log"
