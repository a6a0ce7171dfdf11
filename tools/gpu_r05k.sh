#!/bin/bash
# round 5 checkpoint (part 1): GPU suite, smoke, bench lines of the four BASELINE configs
step() { tools/gpu_step.sh "$@" || exit 1; }
step r05k_pytest 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step r05k_smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
step r05k_bench 300 python -u bench.py
step r05k_bench_c2 300 python -u bench.py --config c2
step r05k_bench_c5 300 python -u bench.py --config c5
echo all-done
