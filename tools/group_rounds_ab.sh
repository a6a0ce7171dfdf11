#!/bin/bash
# Wave-group refill (top-class order) on smaller launches: C3 shards and C4 per threshold (GPU box).
for t in 12 3 1.5; do
  NART_RQ_GROUP_MIN_ROUNDS=$t timeout -k 10 300 python -u tools/shard_perf.py --ns 2 4 8 --reps 2 > gpurun_out/gr_$t.log 2>&1 || { tail -20 gpurun_out/gr_$t.log; exit 1; }
  echo "[t=$t]"; grep '^{' gpurun_out/gr_$t.log | cut -c1-120
done
for t in 12 3; do
  NART_RQ_GROUP_MIN_ROUNDS=$t timeout -k 10 300 python bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/gr_c4_$t.log 2>&1 || exit 1
  echo "[c4 t=$t] $(tail -n1 gpurun_out/gr_c4_$t.log | cut -c1-160)"
done
