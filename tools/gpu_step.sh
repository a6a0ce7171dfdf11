#!/bin/bash
# GPU box helper: run one step under its own time limit, log to gpurun_out/<name>.log, stop the
# chain on failure (exit status of the step).  Usage: tools/gpu_step.sh <name> <seconds> cmd...
name=$1; secs=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 "$secs" "$@" > "gpurun_out/${name}.log" 2>&1
rc=$?
echo "[$name] rc=$rc"; tail -3 "gpurun_out/${name}.log"
exit $rc
