#!/bin/bash
# One GPU-box pass (repo root): gpu parity tests, smoke, default bench, rocprofv3 stats.
#   tools/gpu_check.sh OUT [skip-tests]
OUT=${1:-gpurun_out/check}
mkdir -p "$OUT"
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
  tail -3 "$OUT/pytest.log"
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
  cat "$OUT/smoke.log"
fi
timeout -k 10 600 python -u bench.py > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
bash tools/profile.sh "$OUT/prof" || exit 1
