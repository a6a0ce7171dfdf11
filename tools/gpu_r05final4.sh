#!/bin/bash
# round 5 final sweep (6): GPU suite, smoke, rocprofv3 passes of the C3 / C5 / C4 / C2 bench steps
# (summarised on the box, so that the bench lines below read them), the four bench lines, the
# one-process mode, per-rank shard timings.
step() { tools/gpu_step.sh "$@" || exit 1; }
step r05k2_pytest 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step r05k2_smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
step r05k2_prof_c3 600 bash tools/profile.sh gpurun_out/prof_r05k2_c3
step r05k2_prof_c5 600 bash tools/profile.sh gpurun_out/prof_r05k2_c5 --config c5 --steps 1 --warmup 0 --no-cpu-baseline
step r05k2_prof_c4 900 bash tools/profile.sh gpurun_out/prof_r05k2_c4 --config c4 --steps 1 --warmup 0 --no-cpu-baseline
step r05k2_prof_c2 600 bash tools/profile.sh gpurun_out/prof_r05k2_c2 --config c2 --steps 1 --warmup 0 --no-cpu-baseline
step r05k2_sum 120 bash -c 'python tools/summarize_prof.py gpurun_out/prof_r05k2_c3 r05k2_c3 1920x1080x256 && python tools/summarize_prof.py gpurun_out/prof_r05k2_c5 r05k2_c5 1920x1080x1024 && python tools/summarize_prof.py gpurun_out/prof_r05k2_c4 r05k2_c4 3840x2160x512 && python tools/summarize_prof.py gpurun_out/prof_r05k2_c2 r05k2_c2 1920x1080x64'
step r05k2_bench 300 python -u bench.py
step r05k2_bench_c2 300 python -u bench.py --config c2
step r05k2_bench_c5 300 python -u bench.py --config c5
step r05k2_bench_c4 400 python -u bench.py --config c4 --steps 2
step r05k2_bench_oneproc 300 python -u bench.py --one-process --gpus 1 --no-cpu-baseline
step r05k2_shard_c3 300 python -u tools/shard_perf.py --config c3 --ns 1 2 4 8 --reps 2
step r05k2_shard_c5 300 python -u tools/shard_perf.py --config c5 --ns 1 2 4 8 --reps 2
step r05k2_shard_c4 500 python -u tools/shard_perf.py --config c4 --ns 1 2 4 8 --reps 1
echo all-done
