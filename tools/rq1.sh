# development probe: default-kernel parity subset + timings with env variants (GPU box, repo root):
#   tools/rq1.sh SPP "ENV=..." ...
SPP=$1; shift
mkdir -p gpurun_out/rq1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "rayqueue" > gpurun_out/rq1/parity.log 2>&1; echo "parity rc=$?"; tail -2 gpurun_out/rq1/parity.log
for e in "$@"; do echo "$e"; env $e timeout -k 10 120 python tools/quick_perf.py -s $SPP --reps 2 | tail -1 | cut -c1-100 || exit 1; done
