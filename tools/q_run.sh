#!/bin/bash
# Scheduler experiments (GPU box): tools/q_run.sh LIBNAME [env=val ...]
export NART_HIP_LIB=$PWD/abbuild/$1/libnart_hip.so; shift
mkdir -p gpurun_out/q
timeout -k 10 300 python -u bench.py > gpurun_out/q/bench.log 2>&1 || { tail -20 gpurun_out/q/bench.log; exit 1; }
tail -1 gpurun_out/q/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['parity'])"
for spec in "$@"; do
  env $spec timeout -k 10 300 python -u tools/shard_perf.py --ns 1 2 4 8 --reps 1 > gpurun_out/q/shard.log 2>&1 || { tail -20 gpurun_out/q/shard.log; exit 1; }
  echo "== $spec"; grep '^{' gpurun_out/q/shard.log | python -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print(d['n'], d['worst'])"
done
