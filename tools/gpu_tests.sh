#!/bin/bash
# GPU box: parity suite, then the default bench line (tag = $1).  Every GPU step has its own limit.
set -o pipefail
tag=${1:-run}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_${tag}.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_${tag}.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_${tag}.log 2>&1
tail -2 gpurun_out/bench_${tag}.log
