#!/bin/bash
# round 5 checkpoint 2 (after the triangle-pair / Latin / volume changes): GPU suite, smoke, the
# rocprofv3 passes of C3 / C5 / C4, then the bench lines (which read those summaries only once
# they are copied into profiles/ -- see the second call), shard tables.
step() { tools/gpu_step.sh "$@" || exit 1; }
step r05w_pytest 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step r05w_smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
step r05w_prof_c3 600 bash tools/profile.sh gpurun_out/prof_r05w_c3
step r05w_prof_c5 600 bash tools/profile.sh gpurun_out/prof_r05w_c5 --config c5 --steps 1 --warmup 0 --no-cpu-baseline
step r05w_prof_c4 900 bash tools/profile.sh gpurun_out/prof_r05w_c4 --config c4 --steps 1 --warmup 0 --no-cpu-baseline
echo all-done
