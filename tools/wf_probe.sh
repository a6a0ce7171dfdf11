#!/bin/bash
# Development probe (GPU box, repo root): parity, kernel trace of both variants, SQ counters.
OUT=gpurun_out/${1:-probe}
mkdir -p $OUT
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
cd /tmp && export TMPDIR=/tmp
NART_VARIANT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/kt1 -o run -- python3 $R/tools/quick_perf.py -s 64 --reps 2 > $R/$OUT/kt1.log 2>&1 || exit 1
NART_VARIANT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/kt0 -o run -- python3 $R/tools/quick_perf.py -s 64 --reps 2 > $R/$OUT/kt0.log 2>&1 || exit 1
NART_VARIANT=1 timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAVES --output-format csv -d $R/$OUT/sq1 -o run -- python3 $R/tools/quick_perf.py -s 16 --reps 1 > $R/$OUT/sq1.log 2>&1 || exit 1
NART_VARIANT=0 timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAVES --output-format csv -d $R/$OUT/sq0 -o run -- python3 $R/tools/quick_perf.py -s 16 --reps 1 > $R/$OUT/sq0.log 2>&1 || exit 1
cd $R
grep -h '"' $OUT/kt1.log $OUT/kt0.log | grep samples | cut -c1-300
head -6 $OUT/kt1/run_kernel_stats.csv $OUT/kt0/run_kernel_stats.csv
