#!/bin/bash
# One end-of-round measurement sweep on the GPU box (repo root), every step under its own time
# limit and logged to gpurun_out/<TAG>_<step>.log, stopping at the first failure:
# GPU suite, smoke, rocprofv3 passes (tools/profile.sh) of the four BASELINE configs summarised
# into profiles/ (copied to gpurun_out/<TAG>_profiles/ to come back), then the four bench lines,
# which read those sha-tied summaries.
#   tools/final_sweep.sh TAG [config:WxHxSPP ...]   (default: the four configs)
TAG=${1:?tag}; shift
CONFIGS="$@"; [ -z "$CONFIGS" ] && CONFIGS="c3:1920x1080x256 c5:1920x1080x1024 c2:1920x1080x64 c4:3840x2160x512"
step() { tools/gpu_step.sh "${TAG}_$1" "$2" "${@:3}" || exit 1; }
[ -n "$NO_SUITE" ] || step pytest 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
[ -n "$NO_SUITE" ] || step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
for c in $CONFIGS; do
    name=${c%%:*}; cfg=${c#*:}
    step prof_$name 600 bash tools/profile.sh "gpurun_out/${TAG}_prof_$name" --config $name --steps 1 --warmup 0 --no-cpu-baseline
    step sum_$name 60 python tools/summarize_prof.py "gpurun_out/${TAG}_prof_$name" "${TAG}_$name" $cfg
done
mkdir -p gpurun_out/${TAG}_profiles && cp profiles/${TAG}_* profiles/pmc_latest*.json gpurun_out/${TAG}_profiles/
for c in $CONFIGS; do
    name=${c%%:*}
    if [ $name = c4 ]; then step bench_c4 400 python -u bench.py --config c4 --steps 2
    else step bench_$name 300 python -u bench.py --config $name; fi
done
echo "${TAG} sweep done"
