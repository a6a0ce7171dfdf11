# C3 shard scaling (rank 0 of N) and the other BASELINE configs, one step each (GPU box, repo root)
OUT=${1:-gpurun_out/cfg}
mkdir -p $OUT
timeout -k 10 400 python tools/shard_perf.py --ns 1 2 4 8 --rank 0 > $OUT/shard_c3.log 2>&1 || { tail -5 $OUT/shard_c3.log; exit 1; }
grep "{" $OUT/shard_c3.log
for c in c2 c4 c5; do
  timeout -k 10 400 python -u bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_$c.log 2>&1 || { tail -5 $OUT/bench_$c.log; exit 1; }
  tail -1 $OUT/bench_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['splat_ms_per_step'], d['latin_ms_per_step'])"
done
