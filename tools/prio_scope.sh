#!/bin/bash
# Priority lanes / speculative pairs restricted to small shards: queue parity tests, C3 shards, C4.
OUT=gpurun_out/prio_scope
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "queue" -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 400 python tools/shard_perf.py --config c3 --ns 2 4 8 --reps 2 > $OUT/shard_c3.log 2>&1 || exit 1
tail -n 3 $OUT/shard_c3.log
timeout -k 10 400 python bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_c4.log 2>&1 || exit 1
tail -n 1 $OUT/bench_c4.log | cut -c1-300
