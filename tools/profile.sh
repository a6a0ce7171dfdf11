#!/bin/bash
# rocprofv3 passes over one bench step (run on the GPU box from the repo root):
#   1. kernel trace + stats   2. FETCH_SIZE   3. WRITE_SIZE   4. SQ issue / lane counters
# (separate --pmc passes: FETCH_SIZE and WRITE_SIZE do not fit one pass, MI355X_MICROARCH.md)
# Usage: tools/profile.sh OUT [bench args...]   (default: the C3 bench step)
OUT=${1:-gpurun_out/prof}
shift
ARGS="$@"
[ -z "$ARGS" ] && ARGS="--steps 1 --warmup 0 --no-cpu-baseline"
R=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$R"
run() {  # name, rocprofv3 options...
    local name=$1; shift
    timeout -s KILL 300 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- python3 bench.py $ARGS \
        > "$OUT/$name.log" 2>&1 || { echo "profile pass $name failed"; tail -5 "$OUT/$name.log"; exit 1; }
    echo "pass $name done"
}
run trace --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sq --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_LDS
echo profile-done
