#!/bin/bash
# round 5 final sweep (2), part 1: GPU suite, smoke, rocprofv3 passes of the C3 / C5 / C4 / C2 bench
# steps, and an LDS-counter pass of the C5 bench step (k_splat_skew bank conflicts)
step() { tools/gpu_step.sh "$@" || exit 1; }
step r05ga_pytest 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step r05ga_smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
step r05ga_prof_c3 600 bash tools/profile.sh gpurun_out/prof_r05ga_c3
step r05ga_prof_c5 600 bash tools/profile.sh gpurun_out/prof_r05ga_c5 --config c5 --steps 1 --warmup 0 --no-cpu-baseline
step r05ga_prof_c4 900 bash tools/profile.sh gpurun_out/prof_r05ga_c4 --config c4 --steps 1 --warmup 0 --no-cpu-baseline
step r05ga_prof_c2 600 bash tools/profile.sh gpurun_out/prof_r05ga_c2 --config c2 --steps 1 --warmup 0 --no-cpu-baseline
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES --output-format csv -d $R/gpurun_out/prof_r05ga_c5/lds -o run -- python3 $R/bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/prof_r05ga_c5/lds.log 2>&1 || { echo "lds pass failed"; exit 1; }
echo all-done
