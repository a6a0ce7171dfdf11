#!/bin/bash
# round 5 final sweep, part 1: GPU suite, smoke, rocprofv3 passes of the C3 / C5 / C4 / C2 bench steps
step() { tools/gpu_step.sh "$@" || exit 1; }
step r05fa_pytest 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step r05fa_smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
step r05fa_prof_c3 600 bash tools/profile.sh gpurun_out/prof_r05fa_c3
step r05fa_prof_c5 600 bash tools/profile.sh gpurun_out/prof_r05fa_c5 --config c5 --steps 1 --warmup 0 --no-cpu-baseline
step r05fa_prof_c4 900 bash tools/profile.sh gpurun_out/prof_r05fa_c4 --config c4 --steps 1 --warmup 0 --no-cpu-baseline
step r05fa_prof_c2 600 bash tools/profile.sh gpurun_out/prof_r05fa_c2 --config c2 --steps 1 --warmup 0 --no-cpu-baseline
echo all-done
