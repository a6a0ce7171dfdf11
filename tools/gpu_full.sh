#!/bin/bash
# GPU box: whole parity suite, then the bench lines of every config (tag = $1)
tag=${1:-run}
tools/gpu_step.sh pytest_$tag 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit $?
tools/gpu_step.sh bench_c3_$tag 300 python bench.py --steps 5 --warmup 1 || exit $?
tools/gpu_step.sh bench_c2_$tag 300 python bench.py --config c2 --steps 3 --warmup 1 || exit $?
tools/gpu_step.sh bench_c4_$tag 600 python bench.py --config c4 --steps 2 --warmup 1 || exit $?
tools/gpu_step.sh bench_c5_$tag 300 python bench.py --config c5 --steps 3 --warmup 1 || exit $?
