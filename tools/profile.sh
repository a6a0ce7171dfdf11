#!/bin/bash
# rocprofv3 passes over one bench step (run on the GPU box from the repo root):
#   1. kernel trace + stats   2. FETCH_SIZE   3. WRITE_SIZE   (separate --pmc passes)
set -e
OUT=${1:-gpurun_out/prof}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
ARGS="--steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1
echo profile-done
