#!/bin/bash
# k_splat_skew with two LUT copies (odd lanes on the half-row-shifted copy) vs one.  Splat parity,
# then C5 / C3 whole frames (splat_ms), new vs base, twice; LDS counters of the new C5 step.
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_frames.py -k "splat or skew or c5 or c3" > gpurun_out/r05an_pytest.log 2>&1 || exit 1
L=$R/gpurun_out/r05an_lutc_ab.log
: > $L
for v in new base new base; do
  if [ $v = base ]; then export NART_HIP_LIB=$R/abbuild/lutc1/libnart_hip.so; else unset NART_HIP_LIB; fi
  echo "== $v" >> $L
  timeout -k 10 300 python -u tools/shard_perf.py --config c5 --ns 1 --reps 2 >> $L 2>&1 || exit 1
  timeout -k 10 300 python -u tools/shard_perf.py --config c3 --ns 1 --reps 2 >> $L 2>&1 || exit 1
done
unset NART_HIP_LIB
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES --output-format csv -d $R/gpurun_out/prof_r05an -o run -- python3 $R/bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/prof_r05an.log 2>&1
