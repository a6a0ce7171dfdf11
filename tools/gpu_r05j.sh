#!/bin/bash
# round 5: (1) NART_RQ_HALF + SETPRIO with 12 / 14 / 16 costly pixels per first-round wave, C3 1/8
# shard, all ranks; (2) paired Li_alpha writes (abbuild/pw) vs the default: whole-frame time and
# FETCH_SIZE / WRITE_SIZE of the path kernel
step() { tools/gpu_step.sh "$@" || exit 1; }
step r05j_base 300 python -u tools/shard_perf.py --config c3 --ns 8 --reps 2
for k in 12 14 16; do
  NART_QUEUE_K=$k NART_RQ_HALF=1 NART_RQ_SETPRIO=1 step r05j_hs_k$k 300 python -u tools/shard_perf.py --config c3 --ns 8 --reps 2
done
step r05j_full_def 300 python -u tools/quick_perf.py -s 256 --reps 3
NART_HIP_LIB=abbuild/pw/libnart_hip.so step r05j_full_pw 300 python -u tools/quick_perf.py -s 256 --reps 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in def pw; do
  for c in FETCH_SIZE WRITE_SIZE; do
    if [ $v = pw ]; then export NART_HIP_LIB=abbuild/pw/libnart_hip.so; else unset NART_HIP_LIB; fi
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r05j_pmc_${v}_$c -o run -- python3 tools/quick_perf.py -s 256 --reps 1 > gpurun_out/r05j_pmc_${v}_$c.log 2>&1 || { echo "pmc $v $c failed"; exit 1; }
    echo "pmc $v $c done"
  done
done
echo all-done
