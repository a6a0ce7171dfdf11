# development probe: splat parity tests + splat timing per mode / chunk size (GPU box, repo root)
#   tools/splat_probe.sh SPP "ENV=..." ...
SPP=$1; shift
mkdir -p gpurun_out/splat
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "splat or c1 or high_spp" > gpurun_out/splat/parity.log 2>&1; echo "parity rc=$?"; tail -2 gpurun_out/splat/parity.log
for e in "$@"; do echo "$e"; env $e timeout -k 10 120 python tools/quick_perf.py -s $SPP --reps 2 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('kernel_ms %.2f splat_ms %.2f' % (d['kernel_ms'], d['splat_ms']))" || exit 1; done
