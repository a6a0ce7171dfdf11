#!/bin/bash
# C4 limiter diagnostics: time the env-lit teapot with smaller env maps / constant textures
# (diagnostic scenes, not parity configurations).
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r05n_c4_diag.log
: > $L
run() { echo "== $*" >> $L; timeout -k 10 120 python -u tools/quick_perf.py --scene c4 -w 1920 -H 1080 -s 32 --reps 3 "$@" >> $L 2>&1; }
run && run --env 256 && run --flat rho_d && run --flat roughness && run --flat normal \
  && run --flat rho_d,roughness,normal && run --flat rho_d,roughness,normal --env 256 && run --env 4096
