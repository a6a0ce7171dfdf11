#!/bin/bash
# End-of-round measurement on the GPU box (repo root), each step under its own time limit and
# logged to gpurun_out/<tag>_<step>.log; stops at the first failing step.
#   tools/round_measure.sh TAG part1|part2
#   part1: GPU parity suite, smoke, bench lines of the four BASELINE configs
#   part2: per-rank shard timings (1/2/4/8 ranks) of C3, C5, C4, rocprofv3 passes of the C3 bench
TAG=${1:?tag}; PART=${2:?part}
step() { tools/gpu_step.sh "${TAG}_$1" "$2" "${@:3}" || exit 1; }
if [ "$PART" = part1 ]; then
    DESEL=""
    [ -f tests/golden/frame_c4.npz ] || DESEL="--deselect tests/test_gpu_frames.py::test_whole_frame_matches_oracle_digests[c4]"
    step pytest 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $DESEL
    step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
    step bench 300 python -u bench.py
    step bench_c2 300 python -u bench.py --config c2
    step bench_c5 300 python -u bench.py --config c5
    step bench_c4 400 python -u bench.py --config c4 --steps 2
elif [ "$PART" = part2 ]; then
    step shard_c3 300 python -u tools/shard_perf.py --config c3 --ns 1 2 4 8 --reps 2
    step shard_c5 300 python -u tools/shard_perf.py --config c5 --ns 1 2 4 8 --reps 2
    step shard_c4 500 python -u tools/shard_perf.py --config c4 --ns 1 2 4 8 --reps 1
    step prof 600 bash tools/profile.sh "gpurun_out/prof_${TAG}"
fi
echo "${TAG} ${PART} done"
