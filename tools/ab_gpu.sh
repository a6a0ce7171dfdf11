#!/bin/bash
# One GPU-box A/B pass over prebuilt variants (tools/ab_build.sh): a glassSphere parity subset
# per variant, then kernel timings.  tools/ab_gpu.sh OUT SPP "PYTEST_K" name1 name2 ...
OUT=$1; SPP=$2; K=$3; shift 3
mkdir -p $OUT
for name in "$@"; do
  NART_HIP_LIB=abbuild/$name/libnart_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q \
    --timeout 120 --timeout-method thread -k "$K" > $OUT/parity_$name.log 2>&1 || { echo "PARITY FAIL $name"; tail -20 $OUT/parity_$name.log; exit 1; }
  echo "$name: $(tail -1 $OUT/parity_$name.log)"
done
bash tools/ab_run.sh $SPP "$@" | tee $OUT/timing.log
